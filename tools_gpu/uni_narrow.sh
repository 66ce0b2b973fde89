#!/bin/bash
# Universe shapes: TransE wide (16 floats per lane, spills) vs narrow (8 floats per lane, PT_UNI_NARROW=1), C3 and C4.
set -u
mkdir -p gpurun_out
for w in c4 c3; do
  for n in 0 1; do
    PT_UNI_NARROW=$n PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/un_${w}_$n.log 2>&1 || exit $?
  done
done
