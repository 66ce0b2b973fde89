#!/bin/bash
# Round 5 (v): split-sampler shape sweep on the driver's command (tuning build): threads per part x parts per call
set -u
mkdir -p gpurun_out
T=${TAG:-r05v}
V=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
C="--steps 20 --warmup 5 --no-cpu-baseline --no-c3 --deterministic-timing 0 --repeats 3"
for nt in 256 512 1024; do
  for pc in 8 13 26 52; do
    PT_PART_NT=$nt PT_PART_COUNT=$pc timeout -k 10 300 python tools_gpu/ablib.py $V bench.py $C \
      > gpurun_out/${T}_nt${nt}_pc${pc}.log 2>&1 || exit $?
  done
done
