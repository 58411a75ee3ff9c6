#!/bin/bash
# the GPU round, then the encode ablations (each step time-limited, stop at a failure)
set -u
bash scripts/gpu_round.sh || exit $?
bash scripts/ab_encode.sh
