#!/bin/bash
# same-box A/B of two diagnostic builds of the general decode (phase clock):
# A = iggy_amd/libiggy_codec_diag_old.so, B = iggy_amd/libiggy_codec_diag.so, on C3 and on
# small variable frames (DG_SMALL, default 4 M x U[64, 512] B)
set -u
mkdir -p gpurun_out/ab
for r in 1 2; do
for v in _old ""; do
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag$v.so timeout -k 10 120 python -u scripts/diag_general.py > gpurun_out/ab/c3${v}_$r.log 2>&1 || exit 1
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag$v.so timeout -k 10 120 python -u scripts/diag_general.py ${DG_SMALL:---messages 4194304 --lo 64 --hi 512} > gpurun_out/ab/sm${v}_$r.log 2>&1 || exit 1
done; done
