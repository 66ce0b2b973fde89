#!/bin/bash
# Round 4 (e): fused step + apply diagnostics - fused vs pair rows on one C2 step (product build, and the
# returning-atomics variant ab/lib_ra.so), then the fused parity tests on both builds.
set -u
mkdir -p gpurun_out
T=${TAG:-r04e}
timeout -k 10 300 python tools_gpu/diag_sa.py > gpurun_out/${T}_diag_prod.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/ablib.py ab/lib_ra.so tools_gpu/diag_sa.py > gpurun_out/${T}_diag_ra.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "step_apply or full_size" -m gpu > gpurun_out/${T}_tests_prod.log 2>&1
echo "rc=$?" >> gpurun_out/${T}_tests_prod.log
timeout -k 10 300 python -u tools_gpu/ablib.py ab/lib_ra.so -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "step_apply or full_size" -m gpu > gpurun_out/${T}_tests_ra.log 2>&1
echo "rc=$?" >> gpurun_out/${T}_tests_ra.log
