#!/bin/bash
# Staged-step A/B on the universe workloads: prev = libputranse_hip_prev.so; tuning build with
# PT_UNI_STAGE / PT_UNI_SLOTS off and on.
set -u
mkdir -p gpurun_out
T=${TAG:-st}
R=$PWD/openke-putranse_amd/openke/release
for w in ${WLS:-c3 c5}; do
  PT_UNI_PROF=1 PT_LIB_PATH=$R/libputranse_hip_prev.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}_prev.log 2>&1 || exit $?
  for v in "0 0" "1 0" "1 1"; do
    set -- $v
    PT_UNI_STAGE=$1 PT_UNI_SLOTS=$2 PT_UNI_PROF=1 PT_LIB_PATH=$R/libputranse_hip_tuning.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}_st$1$2.log 2>&1 || exit $?
  done
done
PT_LIB_PATH=$R/libputranse_hip_tuning.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
