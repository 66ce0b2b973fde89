#!/bin/bash
# Round 5 (y): k_lp_scan_t with the abs-modifier adds (product build, 8 waves), C4 kernel statistics twice, then the
# LP / universe tests
set -u
mkdir -p gpurun_out
T=${TAG:-r05y}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0"
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_$i -o run --output-format csv -- \
    python3 bench.py $A > gpurun_out/${T}_c4_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
