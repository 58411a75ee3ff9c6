#!/bin/bash
# Round-4 GPU pass: the whole -m gpu suite, the default bench line, then the
# profile set at this HEAD (scripts/profile_round.sh r04a). Each step under its own
# limit; a failure ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
IGGY_CODEC_DEBUG=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/t3.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench_a.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench_a.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile_round.sh r04a
