#!/bin/bash
# Round 4: universe parity tests on the product build, then a same-box A/B of universe builds (ab_libs.sh).
set -u
mkdir -p gpurun_out
T=${TAG:-r04}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_configs.py tests/test_gpu_ordered.py -m gpu > gpurun_out/${T}_unitests.log 2>&1 || exit $?
TAG=$T LIBS="${LIBS:-base prod}" WLS="${WLS:-c3 c4 c5}" bash tools_gpu/ab_libs.sh || exit $?
# the drop-in universe path (Parallel_Universe_Config as the experiments drive it), product build
for w in ${DWLS:-c3 c4}; do
  timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_dropin_$w.log 2>&1 || exit $?
done
