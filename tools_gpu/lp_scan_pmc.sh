#!/bin/bash
# k_lp_scan_g on C4 (tuning build): kernel statistics at 4 and 3 waves per SIMD, then SQ / LDS counters of each.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-lpgp}
LIB=openke-putranse_amd/openke/release/libputranse_hip_lpv.so
for w in 4 3; do
  PT_LP_G_W=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_w$w -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $LIB bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_w$w.log 2>&1 || exit $?
  PT_LP_G_W=$w timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU \
    -d gpurun_out/${T}_pmc_w$w -o run --output-format csv -- python3 tools_gpu/ablib.py $LIB bench.py --workload c4 --steps 1 \
    --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_pmc_w$w.log 2>&1 || exit $?
done
