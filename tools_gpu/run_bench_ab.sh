#!/bin/bash
# A/B bench variants (CSR vs atomic path) in one GPU call; stops on fault/timeout.
set -u
mkdir -p gpurun_out
for v in 1 0; do
    PT_CSR=$v timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_csr$v.log 2>&1
    rc=$?
    echo "bench_csr$v rc=$rc" >> gpurun_out/steps.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
