#!/bin/bash
# Round 6 (f): team universes with relation partials (tests first), then same-box A/B of C4 on one GPU (round-5
# library, this build, this build with one-row list walks), then C4 / C3 8-way shares with teams (widths 4 and 1).
set -u
mkdir -p gpurun_out
T=${TAG:-r06f}
R5=openke-putranse_amd/openke/release/libputranse_hip_r5.so
LB1=openke-putranse_amd/openke/release/libputranse_hip_lb1.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pu.py -m gpu \
  -k "team" > gpurun_out/${T}_teams.log 2>&1 || exit $?
for k in 1 2; do
  for lib in r5 new lb1; do
    case $lib in
      r5) pre="python tools_gpu/ablib.py $R5 bench.py" ;;
      lb1) pre="python tools_gpu/ablib.py $LB1 bench.py" ;;
      *) pre="python bench.py" ;;
    esac
    timeout -k 10 300 $pre --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
      --deterministic-timing 0 > gpurun_out/${T}_c4_${lib}_$k.log 2>&1 || exit $?
  done
done
for w in c4 c3; do
  for tw in 4 1; do
    timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --team-width $tw \
      --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_${w}_p8_w$tw.log 2>&1 || exit $?
  done
done
