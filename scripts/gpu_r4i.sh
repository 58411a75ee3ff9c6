#!/bin/bash
# General-walk verify through LDS rings: parity of the walk-heavy GPU tests, then a
# same-box A/B of the C3 decode against the previous library (LIBS).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4i
mkdir -p $O
cd $R
export GPU_PINNED_MIN_XFER_SIZE=1048576
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_robust_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_libs.py $LIBS --c3 --rounds ${ROUNDS:-6} > $O/ab_c3.log 2>&1
rc=$?; echo "ab rc=$rc" >> $O/ab_c3.log; exit $rc
