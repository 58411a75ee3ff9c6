set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c3
mkdir -p $O
timeout -k 10 120 python -u scripts/diag_general.py > $O/diag_general.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/enc -o enc -- python3 $R/scripts/bench_encode.py --steps 10 > $O/enc.log 2>&1 || exit $?
