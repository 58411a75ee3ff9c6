#!/bin/bash
# Locate's walk with register-buffered list stores: parity of the walk-heavy GPU tests,
# then a same-box A/B of the C3 decode across LOC_BUF builds (LIBS) and the phase clock.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4j
mkdir -p $O
cd $R
export GPU_PINNED_MIN_XFER_SIZE=1048576
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_robust_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_libs.py $LIBS --c3 --rounds ${ROUNDS:-6} > $O/ab_c3.log 2>&1
rc=$?; echo "ab rc=$rc" >> $O/ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/diag_general.py > $O/diag_general.log 2>&1
rc=$?; echo "diag rc=$rc" >> $O/diag_general.log; exit $rc
