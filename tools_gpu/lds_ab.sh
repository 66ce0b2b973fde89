#!/bin/bash
# LDS budget A/B on the universe workloads: prev build, tuning build at 79 KB (round 2's plan) and at the
# default (the CU's whole LDS).
set -u
mkdir -p gpurun_out
T=${TAG:-lb}
R=$PWD/openke-putranse_amd/openke/release
for w in ${WLS:-c3 c4 c5}; do
  PT_LIB_PATH=$R/libputranse_hip_prev.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}_prev.log 2>&1 || exit $?
  PT_UNI_LDS_KB=79 PT_LIB_PATH=$R/libputranse_hip_tuning.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}_79.log 2>&1 || exit $?
  PT_LIB_PATH=$R/libputranse_hip_tuning.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}_full.log 2>&1 || exit $?
done
