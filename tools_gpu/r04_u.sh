#!/bin/bash
# Round 4 (u): the C3 and C4 sets' schedules (every universe's start / duration and phase cycles) for the CU-share model
set -u
mkdir -p gpurun_out
for w in c3 c4; do
  PT_UNI_PROF=1 PT_UNI_PROF_DUMP=gpurun_out/r04u_sched_$w.npz timeout -k 10 300 python bench.py --workload $w --steps 2 \
    --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/r04u_$w.log 2>&1 || exit $?
done
