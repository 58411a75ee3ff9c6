set -u
cd $GRAFT_REPO_ROOT
STEPS="tests" bash scripts/gpu_round.sh r5g || exit $?
LIBS="ab/lib_m1.so ab/lib_m2.so" ROUNDS=8 bash scripts/gpu_ab.sh || exit $?
mkdir -p gpurun_out/diag5
IGGY_DIAG_LIB=ab/diag_m2.so DIAG_VARIANTS=512,513 timeout -k 10 200 python3 -u scripts/diag_decode.py > gpurun_out/diag5/m2.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5g/iso -o iso -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --no-cpu --no-extra --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r5g/iso.log 2>&1
