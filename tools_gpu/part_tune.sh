#!/bin/bash
# k_sample_part tuning at the driver's K=20: threads per workgroup x parts per call; parity tests first.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampling.py \
    > gpurun_out/pytest_sampling.log 2>&1 || exit $?
for nt in 256 512 1024; do
  for pc in 13 26 52; do
    PT_PART_NT=$nt PT_PART_COUNT=$pc timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/tune_nt${nt}_pc${pc}.log 2>&1 || exit $?
  done
done
