#!/bin/bash
# Same-box A/B of C3 encode library builds with the output check off (bench_encode.py
# --no-check), for the timing-only store ablations of DESIGN.md 4.4: build each variant
# with its knob (IGGY_ER_NOSTORE, IGGY_ER_A128, IGGY_ER_TSTORE, IGGY_ER_MODE=3,
# IGGY_ER_WAVES=8 IGGY_ER_SLOTS=2) into ab/, then LIBS="ab/lib_a.so ab/lib_b.so".
set -u
mkdir -p gpurun_out/era
rm -f gpurun_out/era/summary.log
for r in 1 2 3; do for lib in ${LIBS:-ab/lib_base.so ab/lib_tst.so}; do
  IGGY_DIAG_LIB=$lib timeout -k 10 120 python3 -u scripts/bench_encode.py --steps 10 --no-check > gpurun_out/era/run.log 2>&1 || { cat gpurun_out/era/run.log; exit 1; }
  echo "$lib $(grep '^{' gpurun_out/era/run.log | tail -1)" >> gpurun_out/era/summary.log
done; done
