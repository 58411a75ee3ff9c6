#!/bin/bash
# GPU-box runner (diagnostic): tests -> bench -> rocprofv3 kernel trace of isolated decodes.
# Every GPU step has its own time limit; a step that crashes, hangs or times out
# ends the script (no further GPU step runs).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
TESTS=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u $R/bench.py > $O/b.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/b.log
[ $rc -eq 0 ] || exit $rc
[ "${PROF:-1}" = "1" ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o iso -- python3 $R/bench.py --streams 1 --no-cpu --no-extra --steps 20 > $O/p.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> $O/p.log
exit $rc
