#!/bin/bash
# Round-4 first GPU call: the -m gpu suite without the encryption module (hot-path
# parity first), then the decrypt-fault diagnostic with serialised kernels under a
# kernel trace. A GPU fault or time limit in step 1 ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    --ignore=tests/test_crypt_gpu.py > $O/t1.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t1.log
if [ $rc -gt 1 ] || grep -qiE "illegal|memory access fault|hipErrorLaunch" $O/t1.log; then exit $rc; fi
export AMD_SERIALIZE_KERNEL=3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/crypt -o crypt -- python3 -u scripts/diag_crypt_fault.py > $O/crypt.log 2>&1
rc2=$?; echo "diag rc=$rc2" >> $O/crypt.log
exit $rc2
