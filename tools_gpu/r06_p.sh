#!/bin/bash
# Round 6 (p): the register-blocked TransE LP scan (k_lp_scan_r) - the GPU tests that score link prediction, then
# C4 with kernel stats against the build with k_lp_scan_t (PT_LP_SCAN_R=0): scan time and rank digests.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r06p}
LPT=openke-putranse_amd/openke/release/libputranse_hip_lpt.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_realscale.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu \
  > gpurun_out/${T}_lp_tests.log 2>&1 || exit $?
for lib in new lpt; do
  pre="python3 bench.py"
  [ $lib = lpt ] && pre="python3 tools_gpu/ablib.py $LPT bench.py"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_$lib -o run --output-format csv -- $pre \
    --workload c4 --steps 1 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
    > gpurun_out/${T}_c4_$lib.log 2>&1 || exit $?
done
