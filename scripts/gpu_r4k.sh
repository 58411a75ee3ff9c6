#!/bin/bash
# Round-end check: the whole -m gpu suite, smoke(), the bench line and the C3 phase clock.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4k
mkdir -p $O
cd $R
export GPU_PINNED_MIN_XFER_SIZE=1048576
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/diag_general.py > $O/diag_general.log 2>&1
