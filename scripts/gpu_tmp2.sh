set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/dbg_async.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
