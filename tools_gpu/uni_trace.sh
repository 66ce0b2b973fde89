#!/bin/bash
# Phase stamps of one step of the longest universe (measurement build, PT_UNI_PROF=1) for C3 / C4 / C5.
set -u
mkdir -p gpurun_out
T=${TAG:-tr}
R=$PWD/openke-putranse_amd/openke/release
for w in ${WLS:-c3 c4 c5}; do
  PT_UNI_PROF=1 PT_LIB_PATH=$R/libputranse_hip_tuning.so timeout -k 10 200 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
