#!/bin/bash
# Universe trainer A/B: GPU universe tests, then C3 / C5 lines with phase cycles (PT_UNI_PROF=1), default vs
# 1024-thread workgroups with narrow shapes (PT_UNI_NT=1024).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py > gpurun_out/pytest_pu.log 2>&1 || exit $?
for w in c3 c5; do
  PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/uab_${w}_def.log 2>&1 || exit $?
  PT_UNI_NT=1024 PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/uab_${w}_nt1024.log 2>&1 || exit $?
done
