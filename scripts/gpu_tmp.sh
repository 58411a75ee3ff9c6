set -u
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/encab/summary.log
LIBS="ab/lib_ns.so ab/lib_u8.so ab/lib_u16.so ab/lib_u32.so" bash scripts/gpu_encab.sh && cat gpurun_out/encab/summary.log
