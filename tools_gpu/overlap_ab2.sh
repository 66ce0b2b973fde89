#!/bin/bash
# Overlapped sampling: first-chunk size sweep (2 chunks) at K=20, and grow vs fixed at K=200.
set -u
mkdir -p gpurun_out
run() { local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 $ARGS > gpurun_out/ov2_$name.log 2>&1 || exit $?; }
ARGS="--steps 20 --warmup 5"
run off_k20 PT_OVERLAP=0
for f in 1 2 4; do run f${f}_k20 PT_OVERLAP_FIRST=$f; done
run f2part_k20 PT_OVERLAP_FIRST=2 PT_SAMPLE_MODE=part
ARGS="--steps 200 --warmup 20"
run off_k200 PT_OVERLAP=0
run f2_k200 PT_OVERLAP_FIRST=2
run f2part_k200 PT_OVERLAP_FIRST=2 PT_SAMPLE_MODE=part
