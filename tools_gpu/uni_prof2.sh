#!/bin/bash
# Universe trainer phase cycles (PT_UNI_PROF=1) for C3, C4 and C5.
set -u
mkdir -p gpurun_out
for w in c3 c4 c5; do
  PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/uprof_$w.log 2>&1 || exit $?
done
