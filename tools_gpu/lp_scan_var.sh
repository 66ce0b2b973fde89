#!/bin/bash
# Measurement variants of the DV = 200 TransE LP scan (tuning build, PT_LP_V_VARIANT 0..3) on C4, rocprofv3
# kernel statistics each; then SQ counters of variant 0.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-lpv}
LIB=openke-putranse_amd/openke/release/libputranse_hip_lpv.so
for v in 0 1 2 3; do
  PT_LP_V_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_v$v -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $LIB bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_v$v.log 2>&1 || exit $?
done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  -d gpurun_out/${T}_pmc -o run --output-format csv -- python3 tools_gpu/ablib.py $LIB bench.py --workload c4 --steps 1 \
  --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_pmc.log 2>&1 || exit $?
