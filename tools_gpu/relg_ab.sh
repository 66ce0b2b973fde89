#!/bin/bash
# Relation gradient rows in LDS (float atomics) vs as contribution lists, universe workloads (tuning build).
set -u
mkdir -p gpurun_out
T=${TAG:-rg}
R=$PWD/openke-putranse_amd/openke/release
for w in ${WLS:-c3 c4 c5}; do
  for v in 1 0; do
    PT_UNI_RELGRAD=$v PT_UNI_PROF=1 PT_LIB_PATH=$R/libputranse_hip_tuning.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}_$v.log 2>&1 || exit $?
  done
done
