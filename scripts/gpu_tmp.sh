set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/c1_timing.py 2>&1 | grep -v amdgpu.ids
