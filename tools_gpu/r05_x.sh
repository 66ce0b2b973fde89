#!/bin/bash
# Round 5 (x): k_lp_scan_t at 8 waves with 2 vs 4 pairs per pass (tuning builds), C4 kernel statistics
set -u
mkdir -p gpurun_out
T=${TAG:-r05x}
R=openke-putranse_amd/openke/release
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0"
for v in tuning tuning_p4; do
  PT_LP_WAVES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_$v -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $R/libputranse_hip_$v.so bench.py $A > gpurun_out/${T}_c4_$v.log 2>&1 || exit $?
done
