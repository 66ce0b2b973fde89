#!/bin/bash
# Round 5 (b): the table-driven presampler build - GPU suite (forward-error log at KAPPA_C = 0.5) and the universe
# lines with per-universe phase cycles (PT_UNI_PROF=1: presample / phase A / phase B per step).
set -u
mkdir -p gpurun_out
T=${TAG:-r05b}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 300 python -u -m pytest -q --timeout 120 \
  --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log; [ $rc -le 1 ] || exit $rc
for w in c3 c4 c5; do
  PT_UNI_PROF=1 timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
