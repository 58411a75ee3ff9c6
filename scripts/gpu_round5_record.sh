#!/bin/bash
# The round-5 record run at 89526f5: the round check, the bench with 3 / 4
# pipelined lanes, profiles (trace, C3 phase clock, PMC), and a same-box A/B of two builds.
set -u
cd $GRAFT_REPO_ROOT
STEPS="tests smoke bench phase" bash scripts/gpu_round.sh r5o || exit $?
for k in 3 4; do
timeout -k 10 300 python -u bench.py --streams $k --no-extra --no-cpu > gpurun_out/r5o/bench_s$k.log 2>&1 || exit $?
done
bash scripts/profile_round.sh r05c || exit $?
bash scripts/c3_profile.sh || exit $?
bash scripts/enc_pmc.sh || exit $?
LIBS="ab/lib_head.so ab/lib_lv.so" ROUNDS=6 bash scripts/gpu_ab.sh; tail -4 gpurun_out/ab/abn.log
