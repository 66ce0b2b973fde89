#!/bin/bash
# Universe-kernel evaluation: the universe parity tests, then the C3 / C4 / C5 bench lines with the
# per-universe phase cycles (PT_UNI_PROF=1 makes bench.py enable pt_universe_set_profiling).
set -u
mkdir -p gpurun_out
T=${TAG:-ue}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_ordered.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
for w in c3 c4 c5; do
  PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
