#!/bin/bash
# universe kernel cycle split (PT_UNI_PROF=1) for C3 and C5
set -u
mkdir -p gpurun_out
for wl in c3 c5; do
    echo "== $wl" >> gpurun_out/uni_prof.log
    PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/uni_prof.log 2>&1 || exit $?
done
