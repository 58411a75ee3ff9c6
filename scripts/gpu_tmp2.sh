set -u
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/encab/summary.log
LIBS="ab/lib_ernt0.so ab/lib_ernt1.so" bash scripts/gpu_encab.sh && cat gpurun_out/encab/summary.log | sed 's/"config".*"encode_ms"/encode_ms/; s/, "encode_gib_s.*hbm_frac/ hbm_frac/'
