set -u
cd $GRAFT_REPO_ROOT
for r in 1 2; do for lib in ab/lib_ns.so ab/lib_bs.so ab/lib_bsn.so; do
IGGY_DIAG_LIB=$lib timeout -k 10 120 python3 -u scripts/bench_encode.py --steps 10 --no-check 2>&1 | grep '^{' | sed "s#^#$lib #"
done; done
