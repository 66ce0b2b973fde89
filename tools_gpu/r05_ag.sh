#!/bin/bash
# Round 5 (ag): k_lp_scan_t's TransE tile staged and normalized by 8-lane teams (product build) vs the flat-index
# load + per-lane norms + wave-0 scaling (PT_LP_TEAM=0 build), same box, C4 kernel statistics twice each; LP tests
set -u
mkdir -p gpurun_out
T=${TAG:-r05ag}
R=openke-putranse_amd/openke/release
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0"
for i in 1 2; do
  for v in hip hip_noteam; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_${v}_$i -o run --output-format csv -- \
      python3 tools_gpu/ablib.py $R/libputranse_$v.so bench.py $A > gpurun_out/${T}_c4_${v}_$i.log 2>&1 || exit $?
  done
done
