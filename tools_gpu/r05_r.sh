#!/bin/bash
# Round 5 (r): cProfile of the 512-universe drop-in leg, and the 6,000-universe reference-scale drop-in with the
# GPU-drawn initial tables
set -u
mkdir -p gpurun_out
T=${TAG:-r05r}
timeout -k 10 300 python tools_gpu/prof_dropin.py c3 > gpurun_out/${T}_prof_c3.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c3 --universes 6000 --dim 20 --valid-steps 100 --link-prediction \
  --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_c3_6000.log 2>&1 || exit $?
