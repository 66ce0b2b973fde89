#!/bin/bash
# 128-B aligned contribution rows vs stride dim: GPU tests, then interleaved C2 lines at K=200 and K=20.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for rep in 1 2; do
  for pad in 1 0; do
    PT_CROW_PAD=$pad timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/pad${pad}_k200_$rep.log 2>&1 || exit $?
    PT_CROW_PAD=$pad timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/pad${pad}_k20_$rep.log 2>&1 || exit $?
  done
done
