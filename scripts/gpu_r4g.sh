#!/bin/bash
# Ablation of the C2 uniform decode's roles at this HEAD (diagnostic build):
# 0 full, 1 chain off, 129 chain off + no publishing, 65 chain off + staging only,
# 512 progress stamps. One process, one record, variants interleaved.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abl
mkdir -p $O
cd $R
export GPU_PINNED_MIN_XFER_SIZE=1048576
DIAG_VARIANTS=${VARIANTS:-0,1,129,65,512} timeout -k 10 300 python -u scripts/diag_decode.py > $O/diag.log 2>&1
rc=$?; echo "diag rc=$rc" >> $O/diag.log; exit $rc
