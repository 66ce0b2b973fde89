#!/bin/bash
# Round 4 (l): link-prediction fold launched per row shape instead of per dim - the universe / LP parity tests,
# then the C3 and C4 lines with their drop-in legs (validation and run_link_prediction times).
set -u
mkdir -p gpurun_out
T=${TAG:-r04l}
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in c3 c4; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 \
    > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
