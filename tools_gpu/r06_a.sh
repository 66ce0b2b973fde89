#!/bin/bash
# Round 6 start: the GPU suite on a fresh box (forward-error log), the C4 line with per-universe phase cycles and
# its 8-way placement shares (the chain the round attacks).
set -u
mkdir -p gpurun_out
T=${TAG:-r06a}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 300 python -u -m pytest -q --timeout 120 \
  --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PT_UNI_PROF=1 timeout -k 10 400 python bench.py --workload c4 --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
  --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c4.log 2>&1 || exit $?
PT_UNI_PROF=1 timeout -k 10 400 python bench.py --workload c5 --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
  --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c5.log 2>&1 || exit $?
PT_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  --deterministic-timing 0 --no-ref-scale > gpurun_out/${T}_dist2.log 2>&1 || exit $?
