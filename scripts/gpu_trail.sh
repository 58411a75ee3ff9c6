#!/bin/bash
# C3 encode A/B: the product ring encode (diag build) against the trailing-copier
# prototype (IGGY_ENC_TRAIL: the ring hashes only, a copier kernel on its own stream
# writes the frame bytes), copier grid x1/x2/x4 (IGGY_CODEC_DBG bits 24-27), each run
# checked by a Verify decode of its output (scripts/bench_encode.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trail
mkdir -p $O
cd $R
for r in 1 2; do
  for cfg in "ab/lib_diag_base.so 0" "ab/lib_trail.so 67108864" "ab/lib_trail.so 134217728" "ab/lib_trail.so 251658240"; do
    set -- $cfg
    IGGY_DIAG_LIB=$1 IGGY_CODEC_DBG=$2 timeout -k 10 120 python3 -u scripts/bench_encode.py --steps 10 > $O/run.log 2>&1 || { cat $O/run.log; exit 1; }
    echo "$1 dbg=$2 $(grep '^{' $O/run.log | tail -1)" >> $O/summary.log
  done
done
