#!/bin/bash
# Round 6 (b): the GPU suite on the build with the chain-profile words (forward-error log with the largest error's
# detail), the same teacher-forced C4 / C5 / C3 workload tests on a build whose wide rows take IEEE sqrt / division
# (PT_UNI_FAST_WIDE=0), and the C4 / C3 lines with the chain roofline and their 8-way shares.
set -u
mkdir -p gpurun_out
T=${TAG:-r06b}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 300 python -u -m pytest -q --timeout 120 \
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
for w in c4 c3; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
    --no-dropin --deterministic-timing 0 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
timeout -k 10 400 python tools_gpu/ablib.py openke-putranse_amd/openke/release/libputranse_hip_ieeewide.so bench.py \
  --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
  > gpurun_out/${T}_c4_ieee.log 2>&1 || exit $?
