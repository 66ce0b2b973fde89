#!/bin/bash
# k_sample_part phase timestamps at K=20 (default parts): search on / off (PT_PART_DBG=1, timing only).
set -u
mkdir -p gpurun_out
for d in 0 1; do
  PT_PART_DBG=$d PT_PART_PROF=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/pdbg2_$d.log 2>&1 || exit $?
done
