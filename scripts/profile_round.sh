#!/bin/bash
# GPU-box profile collection (diagnostic): isolated one-lane kernel trace of the
# C2 bench plus separate rocprofv3 --pmc passes (one counter group per run, each
# under its own kill timeout, MI355X_MICROARCH.md "rocprofv3 PMC slots").
# usage: bash scripts/profile_round.sh <tag>   -> gpurun_out/prof_<tag>/
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_${1:-r}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --streams 1 --no-cpu --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/iso -o iso -- python3 $B --steps 20 --warmup 3 > $O/iso.log 2>&1
rc=$?; echo "iso rc=$rc" >> $O/iso.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format rocpd csv -d $O/pmc1 -o pmc -- python3 $B --steps 5 --warmup 2 > $O/pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc" >> $O/pmc1.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format rocpd csv -d $O/pmc2 -o pmc -- python3 $B --steps 5 --warmup 2 > $O/pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc" >> $O/pmc2.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format rocpd csv -d $O/pmc3 -o pmc -- python3 $B --steps 5 --warmup 2 > $O/pmc3.log 2>&1
rc=$?; echo "pmc3 rc=$rc" >> $O/pmc3.log
exit $rc
