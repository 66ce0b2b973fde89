#!/bin/bash
# Universe tests + C3 / C4 / C5 lines with phase cycles.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py > gpurun_out/pytest_pu.log 2>&1 || exit $?
for w in c3 c4 c5; do
  PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/uc_$w.log 2>&1 || exit $?
done
