#!/bin/bash
# Round 4 (b): GPU suite on the product build (kappa-bound calibration log), universe A/B prod vs 1024-thread
# class kernels, the drop-in universe path, the 8-way placement shares of C3.
set -u
mkdir -p gpurun_out
T=${TAG:-r04b}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1 || exit $?
TAG=$T LIBS="${LIBS:-prod nt1024}" WLS="${WLS:-c3 c4 c5}" bash tools_gpu/ab_libs.sh || exit $?
for w in c3 c4; do
  timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_dropin_$w.log 2>&1 || exit $?
done
PT_UNI_PROF=1 timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --place-world 8 > gpurun_out/${T}_place8.log 2>&1 || exit $?
