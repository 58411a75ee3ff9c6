#!/bin/bash
# The round-6 closing record: the round check (tests, smoke, bench, C3
# phase clock), the C2 isolated trace and PMC passes, the C3 encode trace, and the
# C3 encode / decode PMC passes -- every step under its own time limit, the first
# failure ends the script.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r6f}
STEPS="tests smoke bench phase" bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/profile_round.sh r0${TAG#r} || exit $?
bash scripts/c3_profile.sh || exit $?
bash scripts/enc_pmc.sh || exit $?
