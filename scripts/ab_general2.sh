#!/bin/bash
# same-box A/B of the general verify loop (diagnostic build, phase clock):
# 0 = product form, 524288 = no realignment loads (hash wrong: timing only),
# 1048576 = realignment dwords moved from the neighbouring lane with DPP (exact)
set -u
mkdir -p gpurun_out/abg
for r in 1 2; do
for b in 0 524288 1048576; do
  IGGY_DIAG_LIB=iggy_amd/libiggy_codec_diag.so IGGY_CODEC_DBG=$b timeout -k 10 120 python -u scripts/diag_general.py > gpurun_out/abg/g${b}_$r.log 2>&1 || exit 1
done; done
