#!/bin/bash
# GPU-box diagnostic: rocprofv3 PMC passes over the C3 encode (one counter group per run).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/encpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/scripts/bench_encode.py --steps 3 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/p1 -o pmc -- python3 $B > $O/p1.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p2 -o pmc -- python3 $B > $O/p2.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p3 -o pmc -- python3 $B > $O/p3.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR --output-format csv -d $O/p4 -o pmc -- python3 $B > $O/p4.log 2>&1
