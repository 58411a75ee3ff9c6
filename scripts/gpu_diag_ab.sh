#!/bin/bash
# Same-box role ablations of the uniform decode for two diagnostic builds (DLIBS, space
# separated): scripts/diag_decode.py with DIAG_VARIANTS per build -> gpurun_out/diag/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/diag
mkdir -p $O
cd $R
for lib in $DLIBS; do
  b=$(basename $lib .so)
  IGGY_DIAG_LIB=$lib timeout -k 10 200 python3 -u scripts/diag_decode.py > $O/$b.log 2>&1 || exit $?
done
