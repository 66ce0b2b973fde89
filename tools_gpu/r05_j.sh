#!/bin/bash
# Round 5 (j): pairs per LDS pass of the transposed LP scan: 4 (this build) vs 2 and 8 (same box), C4 kernel stats
set -u
mkdir -p gpurun_out
T=${TAG:-r05j}
R=openke-putranse_amd/openke/release
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0"
for v in hip hip_p2 hip_p8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_$v -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $R/libputranse_$v.so bench.py $A > gpurun_out/${T}_c4_$v.log 2>&1 || exit $?
done
