#!/bin/bash
# A/B: fused LDS sample+sort vs the two-pass sampling form on C2, then the GPU parity suite.
set -u
mkdir -p gpurun_out
: > gpurun_out/ss_ab.log
for v in 0 1; do
    echo "== PT_SAMPLE_TWO_PASS=$v" >> gpurun_out/ss_ab.log
    PT_SAMPLE_TWO_PASS=$v timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-c3 >> gpurun_out/ss_ab.log 2>&1
    rc=$?
    echo "rc=$rc" >> gpurun_out/ss_ab.log
    if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/ss_ab.log
exit $rc
