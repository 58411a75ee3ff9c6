#!/bin/bash
# Same-box A/B of the C3 encode between library builds (LIBS), alternating, each run
# checked by a decode of its output (scripts/bench_encode.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/encab
mkdir -p $O
cd $R
for r in 1 2; do
  for lib in $LIBS; do
    IGGY_DIAG_LIB=$lib timeout -k 10 120 python3 -u scripts/bench_encode.py --steps 10 > $O/run.log 2>&1 || { cat $O/run.log; exit 1; }
    echo "$lib $(grep '^{' $O/run.log | tail -1)" >> $O/summary.log
  done
done
