#!/bin/bash
# GPU-box runner (diagnostic): the -m gpu suite, then the general-decode phase clock.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u $R/scripts/diag_general.py ${DG_ARGS:-} > $O/dg.log 2>&1
