#!/bin/bash
# Round-4 record at HEAD: the whole -m gpu suite, the default bench line, the profile
# round (isolated C2 kernel trace + PMC passes), the C3 encode/decode kernel trace and
# the general walk's phase clock. Each GPU step has its own limit; stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-r04b}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile_round.sh $T || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 $R/scripts/bench_encode.py --steps 10 > $O/c3.log 2>&1 || exit $?
timeout -k 10 200 python3 -u $R/scripts/diag_general.py > $O/diag_general.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3pmc1 -o pmc -- python3 $R/scripts/bench_encode.py --steps 3 --warmup 1 > $O/c3pmc1.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/c3pmc2 -o pmc -- python3 $R/scripts/bench_encode.py --steps 3 --warmup 1 > $O/c3pmc2.log 2>&1 || exit $?
exit 0
