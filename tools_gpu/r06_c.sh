#!/bin/bash
# Round 6 (c): team universes first on their own (short limit), then the GPU suite (forward-error log), the
# teacher-forced workload tests on the IEEE-wide build, and the C4 / C3 / C5 lines with their 8-way shares (whose
# per-rank sets take teams: fewer universes than CUs).
set -u
mkdir -p gpurun_out
T=${TAG:-r06c}
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py -m gpu \
  -k "teams" > gpurun_out/${T}_teams.log 2>&1 || exit $?
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 400 python -u -m pytest -q --timeout 120 \
  --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa_ieee.jsonl timeout -k 10 300 python -u tools_gpu/ablib.py \
  openke-putranse_amd/openke/release/libputranse_hip_ieeewide.so -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_gpu_configs.py -m gpu -k "pu_workload" > gpurun_out/${T}_pytest_ieee.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest_ieee.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in c4 c3 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
    --no-dropin --deterministic-timing 0 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
