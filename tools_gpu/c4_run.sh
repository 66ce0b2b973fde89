#!/bin/bash
# PU GPU tests (LP kernels changed), then C4 and C5 bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_pu.py -q -x -p no:cacheprovider > gpurun_out/pu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload c4 --steps 1 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || exit $?
