#!/bin/bash
# same-box A/B of encode variants selected by diagnostic bits (diagnostic build):
# 0 = product form, 16384 = lane-group grid over every CU (no CU left for the chain)
set -u
mkdir -p gpurun_out/abe
for r in 1 2; do
for b in 0 16384; do
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag.so IGGY_CODEC_DBG=$b timeout -k 10 120 python -u scripts/bench_encode.py --steps 20 > gpurun_out/abe/e${b}_$r.log 2>&1 || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/abe/tr -o enc -- python3 $GRAFT_REPO_ROOT/scripts/bench_encode.py --steps 5 > $GRAFT_REPO_ROOT/gpurun_out/abe/tr.log 2>&1
