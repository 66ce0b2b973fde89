#!/bin/bash
# Round 4 (i): the drop-in universe path timed at C3 and C4 scale (train_parallel_universes, run_link_prediction;
# breakdown), the C3 schedule on the 8-float float4 shapes, and the universe parity tests on this build.
set -u
mkdir -p gpurun_out
T=${TAG:-r04i}
PT_UNI_PROF=1 PT_UNI_PROF_DUMP=gpurun_out/${T}_prof_c3.npz timeout -k 10 300 python bench.py --workload c3 --steps 2 \
  --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_c3.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 \
  > gpurun_out/${T}_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
  --deterministic-timing 0 > gpurun_out/${T}_c5.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1
echo "rc=$?" >> gpurun_out/${T}_tests.log
