#!/bin/bash
# GPU tests, k_sample_part phase timestamps (PT_PART_PROF=1) at K=20, and the default K=20/K=200 lines.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for pc in 13 26 52; do
  PT_PART_PROF=1 PT_PART_COUNT=$pc timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/pprof_pc$pc.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/k200.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/k20.log 2>&1 || exit $?
