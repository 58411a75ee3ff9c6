#!/bin/bash
# GPU-box runner (diagnostic): the -m gpu suite only (TESTS= to narrow), one process,
# its own time limit; the log lands in gpurun_out/t.log.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t.log
exit $rc
