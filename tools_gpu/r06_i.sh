#!/bin/bash
# Round 6 (i): L2 warm-ahead in the universe kernel - the universe tests, then same-box A/B against the build
# without it (PT_UNI_WARM=0) on C4, C3, C5, and C4's 8-way shares.
set -u
mkdir -p gpurun_out
T=${TAG:-r06i}
NW=openke-putranse_amd/openke/release/libputranse_hip_nowarm.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py -m gpu \
  > gpurun_out/${T}_pu_tests.log 2>&1 || exit $?
for k in 1 2; do
  for w in c4 c3 c5; do
    [ $k = 2 ] && [ $w != c4 ] && continue
    timeout -k 10 300 python tools_gpu/ablib.py $NW bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline \
      --no-dropin --deterministic-timing 0 > gpurun_out/${T}_${w}_nowarm_$k.log 2>&1 || exit $?
    timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
      --deterministic-timing 0 > gpurun_out/${T}_${w}_warm_$k.log 2>&1 || exit $?
  done
done
timeout -k 10 400 python bench.py --workload c4 --steps 2 --warmup 1 --place-world 8 --team-width 1 \
  --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c4_p8.log 2>&1 || exit $?
