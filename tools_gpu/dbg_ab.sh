#!/bin/bash
# C2 step-kernel ablations (PT_STEP_DBG bits: 1 no contrib stores, 2 no positive atomics, 4 no negative-row loads)
set -u
mkdir -p gpurun_out
for v in ${DBG_SET:-0 8 15}; do
    echo "== dbg=$v" >> gpurun_out/dbg_ab.log
    PT_STEP_DBG=$v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 >> gpurun_out/dbg_ab.log 2>&1 || exit $?
done
