#!/bin/bash
# A/B of a candidate decode build against the base build (ab/libbase.so), after the
# candidate's uniform-decode parity tests pass. Each step under its own limit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
export GPU_PINNED_MIN_XFER_SIZE=1048576
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_robust_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_libs.py ${BASE:-ab/libbase.so} iggy_amd/libiggy_codec.so > $O/ab.log 2>&1
rc=$?; echo "ab rc=$rc" >> $O/ab.log; exit $rc
