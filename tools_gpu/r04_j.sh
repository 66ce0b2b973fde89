#!/bin/bash
# Round 4 (j): Python-level profile of the drop-in universe path (C3: train_parallel_universes(512) with its 4
# validations and best-model checkpoints) - where the host time goes.
set -u
mkdir -p gpurun_out
T=${TAG:-r04j}
timeout -k 10 300 python -m cProfile -o gpurun_out/${T}_dropin.pstats bench.py --workload c3 --steps 1 --warmup 1 \
  --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_c3.log 2>&1 || exit $?
