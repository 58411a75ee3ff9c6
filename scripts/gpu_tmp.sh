set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5d
timeout -k 10 120 ./scripts/lat_micro > gpurun_out/r5d/lat_micro.log 2>&1 || exit $?
STEPS="tests bench" bash scripts/gpu_round.sh r5d
