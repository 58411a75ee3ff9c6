#!/bin/bash
# same-box A/B of encode variants selected by diagnostic bits (diagnostic build):
# 0 = product form; 0x10000 = lane-group stores to a 16-B aligned destination (output
# wrong: timing only); 0x20000 = no frame stores; 0x40000 = no hashing; combinations
set -u
mkdir -p gpurun_out/abe
for r in 1 2; do
for b in ${BITS:-0 65536 131072 262144 327680 393216}; do
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag.so IGGY_CODEC_DBG=$b timeout -k 10 120 python -u scripts/bench_encode.py --steps 20 > gpurun_out/abe/e${b}_$r.log 2>&1 || exit 1
done; done
