#!/bin/bash
# Round 6 (e): same-box A/B of C4 on one GPU (round-5 library vs this build, alternating), then this build's C4 / C3
# 8-way shares with the per-share longest universe's team data (width, one XCD, barrier cycles).
set -u
mkdir -p gpurun_out
T=${TAG:-r06e}
R5=openke-putranse_amd/openke/release/libputranse_hip_r5.so
for k in 1 2; do
  timeout -k 10 300 python tools_gpu/ablib.py $R5 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c4_r5_$k.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_c4_new_$k.log 2>&1 || exit $?
done
for w in c4 c3; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
    --no-dropin --deterministic-timing 0 > gpurun_out/${T}_${w}_p8.log 2>&1 || exit $?
done
