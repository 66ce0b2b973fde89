#!/bin/bash
# Round 6 (d): team universes (relation rows through static slots, plain stores when a team shares an XCD) first on
# their own, then the GPU suite (forward-error log), then the C4 / C3 / C5 lines with their 8-way shares.
set -u
mkdir -p gpurun_out
T=${TAG:-r06d}
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py -m gpu \
  -k "teams" > gpurun_out/${T}_teams.log 2>&1 || exit $?
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 400 python -u -m pytest -q --timeout 120 \
  --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in c4 c3 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
    --no-dropin --deterministic-timing 0 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
