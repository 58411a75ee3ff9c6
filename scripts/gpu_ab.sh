#!/bin/bash
# Same-box A/B/C of library builds (LIBS, space separated) on the C2 decode (scripts/ab_libs.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
timeout -k 10 400 python -u scripts/ab_libs.py $LIBS --rounds ${ROUNDS:-6} > $O/abn.log 2>&1
rc=$?; echo "ab rc=$rc" >> $O/abn.log; exit $rc
