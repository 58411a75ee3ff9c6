#!/bin/bash
# GPU-box runner: the whole -m gpu suite, then bench.py, then the multi-record walk
# benchmark; every step under its own time limit, stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u $R/bench.py ${BENCH_ARGS:-} > $O/b.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/b.log; [ $rc -eq 0 ] || exit $rc
[ "${RB:-1}" = "1" ] || exit 0
timeout -k 10 300 python -u $R/scripts/records_bench.py > $O/rb.log 2>&1
rc=$?; echo "records_bench rc=$rc" >> $O/rb.log
exit $rc
