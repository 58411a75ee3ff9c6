#!/bin/bash
# C3 encode ablation (diagnostic build): 0 product behaviour, 0x10000 frame stores to
# 16-B aligned destinations (wrong bytes: the speed of aligned stores), 0x20000 no
# frame stores, 0x40000 no hashing. One process per variant, same seed.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/encabl
mkdir -p $O
cd $R
export GPU_PINNED_MIN_XFER_SIZE=1048576 IGGY_DIAG_LIB=$R/iggy_amd/libiggy_codec_diag.so
for v in 0 65536 131072 262144 0; do
  IGGY_CODEC_DBG=$v timeout -k 10 120 python3 -u scripts/bench_encode.py --steps 10 $( [ $v -ne 0 ] && echo --no-check ) > $O/enc_$v.log 2>&1 || exit $?
  echo "dbg=$v $(grep '^{' $O/enc_$v.log | tail -1)" >> $O/summary.log
done
