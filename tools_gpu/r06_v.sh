#!/bin/bash
# Round 6 (v): phase stamps of one step (epoch 1, step 5) of the longest universe, measurement build (make TUNING=1,
# PT_UNI_PROF=1): C4 / C3 / C5, alone (--longest-only) and in the full set. Dumps in gpurun_out/stamps/.
set -u
mkdir -p gpurun_out/stamps
TL=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
for w in c4 c3 c5; do
  for m in alone set; do
    extra=""
    [ $m = alone ] && extra="--longest-only --team-width 1"
    PT_UNI_PROF=1 PT_UNI_PROF_DUMP=gpurun_out/stamps/${w}_$m.npz timeout -k 10 300 python tools_gpu/ablib.py $TL bench.py \
      --workload $w $extra --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
      > gpurun_out/stamps/${w}_$m.log 2>&1 || exit $?
  done
done
