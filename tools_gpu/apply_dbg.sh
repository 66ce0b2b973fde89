#!/bin/bash
# Step / apply ablations at K=200 (PT_STEP_DBG: 1 no contribution stores, 8 contribution reads from a hot
# 4096-row window, 9 both). Timing only: the results are wrong with any bit set.
set -u
mkdir -p gpurun_out
for d in 0 1 8 9; do
  PT_STEP_DBG=$d timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/adbg_$d.log 2>&1 || exit $?
done
