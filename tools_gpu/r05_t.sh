#!/bin/bash
# Round 5 (t): checkpoint-engine GPU test, then the 6,000-universe reference-scale drop-in and the default line
set -u
mkdir -p gpurun_out
T=${TAG:-r05t}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_checkpoint.py \
  tests/test_gpu_pu.py > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c3 --universes 6000 --dim 20 --valid-steps 100 --link-prediction \
  --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_c3_6000.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${T}_default.log 2>&1 || exit $?
