#!/bin/bash
# LDS-slot entity gradients A/B on the universe workloads (tuning build: PT_UNI_SLOTS=0 / 1), then the
# universe parity tests with slots on.
set -u
mkdir -p gpurun_out
T=${TAG:-sl}
export PT_LIB_PATH=$PWD/openke-putranse_amd/openke/release/libputranse_hip_tuning.so
for w in ${WLS:-c3 c5 c4}; do
  for sl in 0 1; do
    PT_UNI_SLOTS=$sl PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}_s$sl.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
