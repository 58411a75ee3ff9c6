#!/bin/bash
# the GPU round, then the diagnostic candidates: the streamed general decode's parity
# suite and its same-box timing, the encode and general-verify ablations (each step
# time-limited, stop at the first failure)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
bash scripts/gpu_round.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_stream_diag_gpu.py -m gpu_diag -x -v --timeout 240 \
    --timeout-method thread > $O/sd.log 2>&1
rc=$?; echo "stream diag rc=$rc" >> $O/sd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_stream.py > $O/bs_stream.log 2>&1 || exit $?
bash scripts/ab_encode.sh || exit $?
bash scripts/ab_general2.sh
