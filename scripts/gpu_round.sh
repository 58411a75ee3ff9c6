#!/bin/bash
# GPU-box round check: the whole -m gpu suite, smoke(), the bench line, the C3
# general-walk phase clock. Every step under its own time limit; the first failure
# ends the script (no further GPU step runs). usage: bash scripts/gpu_round.sh <tag>
# -> gpurun_out/<tag>/. STEPS narrows it (default "tests smoke bench phase").
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-round}
mkdir -p $O
cd $R
STEPS=${STEPS:-tests smoke bench phase}
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 ;;
    smoke) timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 ;;
    bench) timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 ;;
    phase) timeout -k 10 200 python -u scripts/diag_general.py ${DG_ARGS:-} > $O/phase.log 2>&1 ;;
    records) timeout -k 10 300 python -u scripts/records_bench.py > $O/records.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?; echo "$s rc=$rc" >> $O/steps.log
  [ $rc -eq 0 ] || exit $rc
done
