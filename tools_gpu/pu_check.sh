#!/bin/bash
# PU GPU tests, then the universe cycle split and bench lines for C3 and C5
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pu_tests.log 2>&1 || exit $?
bash tools_gpu/uni_prof.sh || exit $?
if [ "${WITH_C4:-0}" = 1 ]; then
    timeout -k 10 300 python bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit $?
fi
