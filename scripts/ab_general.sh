set -u
mkdir -p gpurun_out/ab
for r in 1 2; do
for v in 0 4 ""; do
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag$v.so timeout -k 10 120 python -u scripts/diag_general.py > gpurun_out/ab/dg${v:-8}_$r.log 2>&1 || exit 1
done; done
