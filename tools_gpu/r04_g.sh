#!/bin/bash
# Round 4 (g): the fused step + apply at 8 waves per SIMD (ab/lib_o8.so, 64 VGPRs) vs the product (fused and pair)
# on the driver-shaped C2 line; then the whole GPU suite on the product build with the forward-error (kappa) log.
set -u
mkdir -p gpurun_out
T=${TAG:-r04g}
for i in 1 2; do
  timeout -k 10 300 python tools_gpu/ablib.py ab/lib_o8.so bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 \
    --no-dropin --step-apply 1 > gpurun_out/${T}_c2_o8_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin --step-apply 1 \
    > gpurun_out/${T}_c2_sa1_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin --step-apply 0 \
    > gpurun_out/${T}_c2_sa0_$i.log 2>&1 || exit $?
done
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 900 python -u -m pytest -q --timeout 300 \
  --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
exit $rc
