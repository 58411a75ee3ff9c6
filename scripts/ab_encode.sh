#!/bin/bash
# same-box A/B of encode variants selected by diagnostic bits (diagnostic build)
set -u
mkdir -p gpurun_out/abe
for r in 1 2; do
for b in 0 4096 8192; do
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag.so IGGY_CODEC_DBG=$b timeout -k 10 120 python -u scripts/bench_encode.py --steps 20 > gpurun_out/abe/e${b}_$r.log 2>&1 || exit 1
done; done
