set -u
cd $GRAFT_REPO_ROOT
STEPS="tests smoke bench phase" bash scripts/gpu_round.sh r5o || exit $?
bash scripts/profile_round.sh r05c || exit $?
bash scripts/c3_profile.sh || exit $?
bash scripts/enc_pmc.sh || exit $?
