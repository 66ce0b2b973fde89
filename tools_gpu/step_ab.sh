#!/bin/bash
# GPU tests, then C2 step-kernel variants (env settings in $VARIANTS, ';'-separated)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit $?
IFS=';' read -ra VS <<< "${VARIANTS:-PT_DUMMY=0}"
for v in "${VS[@]}"; do
    echo "== $v" >> gpurun_out/step_ab.log
    env $v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 >> gpurun_out/step_ab.log 2>&1 || exit $?
done
