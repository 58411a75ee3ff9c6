#!/bin/bash
# the GPU round, then the encode and general-verify ablations (each step
# time-limited, stop at the first failure)
set -u
bash scripts/gpu_round.sh || exit $?
bash scripts/ab_encode.sh || exit $?
bash scripts/ab_general2.sh
