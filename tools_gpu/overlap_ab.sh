#!/bin/bash
# Overlapped sampling schedule: GPU tests, then C2 lines at K=20 / K=200 with the overlap on / off and with
# the split sampler forced for every chunk.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit $?
run() { # name env... -- args
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 $ARGS > gpurun_out/ov_$name.log 2>&1 || exit $?
}
for k in 20 200; do
  w=$(( k / 4 )); [ $w -lt 5 ] && w=5
  ARGS="--steps $k --warmup $w"
  run on_k$k PT_OVERLAP=1
  run off_k$k PT_OVERLAP=0
  run part_k$k PT_OVERLAP=1 PT_SAMPLE_MODE=part
done
