#!/bin/bash
# Base-row form of the C2 step (k_step_csr<BASE> + k_apply_base): GPU tests, then C2 lines with the form on / off.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit $?
run() { local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 $ARGS > gpurun_out/base_$name.log 2>&1 || exit $?; }
for k in 20 200; do
  w=$(( k / 4 )); [ $w -lt 5 ] && w=5
  ARGS="--steps $k --warmup $w"
  run on_k$k PT_STEP_BASE=1
  run off_k$k PT_STEP_BASE=0
done
