#!/bin/bash
# Round 5 (z): k_lp_scan_t base rows through VMEM one group ahead (tuning build) vs scalar loads (tuning build with
# PT_LP_VPREF=0), C4 kernel statistics each, then the LP / universe tests on the tuning build
set -u
mkdir -p gpurun_out
T=${TAG:-r05z}
R=openke-putranse_amd/openke/release
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0"
for v in tuning tuning_nv; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_$v -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $R/libputranse_hip_$v.so bench.py $A > gpurun_out/${T}_c4_$v.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools_gpu/ablib.py $R/libputranse_hip_tuning.so -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
