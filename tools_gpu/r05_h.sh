#!/bin/bash
# Round 5 (h): C4's wide hot kernel at 512 threads (256 VGPRs, no spill, two phase-B rows per lane group) against
# the product's 1,024 threads (128 VGPRs, 136 B of spills), same box, alternating; then the default bench line.
set -u
mkdir -p gpurun_out
T=${TAG:-r05h}
V=openke-putranse_amd/openke/release/libputranse_hip_h512.so
for i in 1 2; do
  PT_UNI_PROF=1 timeout -k 10 300 python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_c4_prod_$i.log 2>&1 || exit $?
  PT_UNI_PROF=1 timeout -k 10 300 python tools_gpu/ablib.py $V bench.py --workload c4 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c4_h512_$i.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py > gpurun_out/${T}_default.log 2>&1 || exit $?
