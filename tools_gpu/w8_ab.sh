#!/bin/bash
# k_step_csr at 8 waves/SIMD vs 7: step parity tests, then interleaved C2 lines at K=20 and K=200.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sampling.py > gpurun_out/pytest_w8.log 2>&1 || exit $?
for rep in 1 2; do
  for w in 1 0; do
    PT_STEP_W8=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/w8_${w}_k20_$rep.log 2>&1 || exit $?
    PT_STEP_W8=$w timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/w8_${w}_k200_$rep.log 2>&1 || exit $?
  done
done
