#!/bin/bash
# Sampling parity tests, the split sampler's phase profile and the K=20 line x2.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampling.py tests/test_gpu_parity.py > gpurun_out/pytest_pq.log 2>&1 || exit $?
PT_PART_PROF=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/pq_prof.log 2>&1 || exit $?
for rep in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/pq_k20_$rep.log 2>&1 || exit $?
done
