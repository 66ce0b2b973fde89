#!/bin/bash
# Round 4 (f): fused step + apply after the carried-flag fix - parity tests, diagnostics, and the driver-shaped
# C2 line: fused (4 waves per positive), fused with at most 2 waves per positive (ab/lib_s2.so), the pair.
set -u
mkdir -p gpurun_out
T=${TAG:-r04f}
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "step_apply or counting_sort or full_size or teacher_forced" -m gpu > gpurun_out/${T}_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools_gpu/diag_sa.py > gpurun_out/${T}_diag.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin --step-apply 1 \
    > gpurun_out/${T}_c2_sa1_$i.log 2>&1 || exit $?
  timeout -k 10 300 python tools_gpu/ablib.py ab/lib_s2.so bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 \
    --no-dropin --step-apply 1 > gpurun_out/${T}_c2_s2_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin --step-apply 0 \
    > gpurun_out/${T}_c2_sa0_$i.log 2>&1 || exit $?
done
