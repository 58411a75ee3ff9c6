#!/bin/bash
# same-box A/B of two diagnostic builds of the uniform decode (scripts/diag_decode.py):
# A = iggy_amd/libiggy_codec_diag_old.so, B = iggy_amd/libiggy_codec_diag.so
set -u
mkdir -p gpurun_out/abu
for r in 1 2; do
for v in _old ""; do
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag$v.so DIAG_VARIANTS=${DIAG_VARIANTS:-0,1} timeout -k 10 200 python -u scripts/diag_decode.py > gpurun_out/abu/u${v}_$r.log 2>&1 || exit 1
done; done
