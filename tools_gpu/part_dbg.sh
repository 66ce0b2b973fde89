#!/bin/bash
# k_sample_part ablations (PT_PART_DBG bits: 1 no run search, 2 no stream jump, 4 no 64-bit modulo) with phase
# timestamps at K=20, 13 parts per call. Timing only: the batches are wrong with any bit set.
set -u
mkdir -p gpurun_out
for d in 0 1 2 4 7; do
  PT_PART_DBG=$d PT_PART_PROF=1 PT_PART_COUNT=13 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/pdbg_$d.log 2>&1 || exit $?
done
