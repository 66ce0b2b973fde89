#!/bin/bash
# k_apply_buf contribution rows in flight per lane group (PT_APPLY_NC 4 vs 8), interleaved, K=200 and K=20.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for nc in 4 8; do
    PT_APPLY_NC=$nc timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/nc${nc}_k200_$rep.log 2>&1 || exit $?
    PT_APPLY_NC=$nc timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/nc${nc}_k20_$rep.log 2>&1 || exit $?
  done
done
