#!/bin/bash
# GPU tests + C2 lines at K=20 (x2) and K=200 (x2).
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for rep in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/q2_k20_$rep.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/q2_k200_$rep.log 2>&1 || exit $?
done
