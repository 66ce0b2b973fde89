#!/bin/bash
# Universe trainer phase cycles (PT_UNI_PROF=1) for C3 and C5.
set -u
mkdir -p gpurun_out
PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/uprof_c3.log 2>&1 || exit $?
PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/uprof_c5.log 2>&1 || exit $?
