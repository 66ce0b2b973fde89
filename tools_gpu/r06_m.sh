#!/bin/bash
# Round 6 (m): per-universe cycle profiles (PT_UNI_PROF dumps) of C4, C3, C5 and of C4's 8-way shares, for the
# set's universe time model (placement, shares, private-L2 choice).
set -u
mkdir -p gpurun_out/dumps
for w in c4 c3 c5; do
  extra=""
  [ $w = c4 ] && extra="--place-world 8"
  PT_UNI_PROF=1 PT_UNI_PROF_DUMP=gpurun_out/dumps/$w.npz timeout -k 10 400 python bench.py --workload $w --steps 1 \
    --warmup 1 $extra --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/dumps/$w.log 2>&1 || exit $?
done
