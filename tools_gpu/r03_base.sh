#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r03_base_pytest.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r03_base_k20.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_base_c3.log 2>&1 || exit $?
