#!/bin/bash
# Round 5 (w): k_lp_scan_t with 4 / 8 / 16 waves per workgroup sharing the tile (tuning build, PT_LP_WAVES),
# C4 kernel statistics each, then the LP tests at 8 and 16 waves
set -u
mkdir -p gpurun_out
T=${TAG:-r05w}
V=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0"
for nw in 4 8 16; do
  PT_LP_WAVES=$nw timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_nw$nw -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $V bench.py $A > gpurun_out/${T}_c4_nw$nw.log 2>&1 || exit $?
done
for nw in 8 16; do
  PT_LP_WAVES=$nw timeout -k 10 300 python -u tools_gpu/ablib.py $V -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_pu.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests_nw$nw.log 2>&1 || exit $?
done
