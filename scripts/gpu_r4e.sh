#!/bin/bash
# Round-4 measurement pass (each step under its own limit; a failure ends the call):
#  1. host-buffer record paths (scripts/records_bench.py) and the decode crossover
#     (scripts/crossover.py) -> GPU_MIN_BYTES of the Rust dispatcher
#  2. the two-lane pipelined C2 run under a kernel trace (the bench's `value` config)
#  3. C3 encode / decode: phase clock (diag_general.py) + kernel traces + PMC passes
#  (4. the streamed-decode candidate, measured once: profiles/r04a_stream_candidate.jsonl, dropped)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/m4
mkdir -p $O
cd $R
export GPU_PINNED_MIN_XFER_SIZE=1048576
timeout -k 10 300 python3 -u scripts/records_bench.py > $O/records.jsonl 2> $O/records.err || exit $?
timeout -k 10 300 python3 -u scripts/crossover.py > $O/crossover.jsonl 2> $O/crossover.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pipe -o pipe -- python3 $R/bench.py --streams 2 --no-cpu --no-extra --steps 20 --warmup 3 > $O/pipe.log 2>&1 || exit $?
timeout -k 10 200 python3 -u $R/scripts/diag_general.py > $O/diag_general.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/enc -o enc -- python3 $R/scripts/bench_encode.py --steps 10 > $O/enc.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/encpmc1 -o pmc -- python3 $R/scripts/bench_encode.py --steps 3 --warmup 1 > $O/encpmc1.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/encpmc2 -o pmc -- python3 $R/scripts/bench_encode.py --steps 3 --warmup 1 > $O/encpmc2.log 2>&1 || exit $?
# (the streamed candidate was measured once here -- profiles/r04a_stream_candidate.jsonl -- and dropped)
exit 0
