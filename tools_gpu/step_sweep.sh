#!/bin/bash
# k_step_csr shape sweep (PT_STEP_NCH x PT_STEP_S) at K=200, default first and last as the drift check.
set -u
mkdir -p gpurun_out
run() { local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/ss_$name.log 2>&1 || exit $?; }
run def0
run nch4 PT_STEP_NCH=4
run nch1 PT_STEP_NCH=1
run s2 PT_STEP_S=2 PT_STEP_NCH=2
run s2n4 PT_STEP_S=2 PT_STEP_NCH=4
run def1
