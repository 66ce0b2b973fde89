#!/bin/bash
# Same-box A/B of two library builds on the universe workloads: A = openke/release/libputranse_hip_prev.so,
# B = the current build; alternated twice (bench.py --workload cX, no CPU baseline).
set -u
mkdir -p gpurun_out
T=${TAG:-ab}
A=$PWD/openke-putranse_amd/openke/release/libputranse_hip_prev.so
for rep in 1 2; do
  for w in ${WLS:-c3 c4 c5}; do
    PT_LIB_PATH=$A timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_A_${w}_$rep.log 2>&1 || exit $?
    timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_B_${w}_$rep.log 2>&1 || exit $?
  done
done
