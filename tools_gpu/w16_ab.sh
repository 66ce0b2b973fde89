#!/bin/bash
# A/B of the 16-float scalar universe shapes (PT_UNI_W16=1) vs 8-float (default) on C3, same box; universe
# parity tests first.
set -u
mkdir -p gpurun_out
PT_UNI_W16=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py -m gpu -k "kernel_matches or training_matches" > gpurun_out/w16_pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload c3 --steps 3 --warmup 1 > gpurun_out/w16_c3_w8_$i.log 2>&1 || exit $?
  PT_UNI_W16=1 timeout -k 10 200 python bench.py --workload c3 --steps 3 --warmup 1 > gpurun_out/w16_c3_w16_$i.log 2>&1 || exit $?
done
PT_UNI_W16=1 PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload c3 --steps 2 --warmup 1 > gpurun_out/w16_c3_prof.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/w16_full_pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/w16_k20.log 2>&1 || exit $?
