#!/bin/bash
# Round 5 (ac): C2 on the current library vs the round-5 closing-evidence library (commit 0dcb6cd), same box,
# interleaved: the driver's 20-step command and the 200-step default shape
set -u
mkdir -p gpurun_out
T=${TAG:-r05ac}
R=openke-putranse_amd/openke/release
C="--no-cpu-baseline --no-c3 --deterministic-timing 0 --repeats 3"
for i in 1 2 3; do
  for v in hip hip_r05close; do
    timeout -k 10 300 python tools_gpu/ablib.py $R/libputranse_$v.so bench.py --steps 20 --warmup 5 $C > gpurun_out/${T}_${v}_k20_$i.log 2>&1 || exit $?
    timeout -k 10 300 python tools_gpu/ablib.py $R/libputranse_$v.so bench.py $C > gpurun_out/${T}_${v}_k200_$i.log 2>&1 || exit $?
  done
done
