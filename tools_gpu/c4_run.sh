#!/bin/bash
# PU GPU tests, then C4 link prediction with different key-batch sizes, C5 with CPU baseline.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_pu.py -q -x -p no:cacheprovider > gpurun_out/pu_tests.log 2>&1 || exit $?
for mb in 192 64 100000; do
    echo "== batch_mb=$mb" >> gpurun_out/bench_c4.log
    PT_LP_BATCH_MB=$mb timeout -k 10 500 python bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/bench_c4.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --workload c5 --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_c5.log 2>&1 || exit $?
