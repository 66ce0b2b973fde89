#!/bin/bash
# Round 5 (an): where the split sampler's slot phase goes at K = 20 - timing ablations of the tuning build
# (PT_PART_DBG bit 0 no run search, bit 1 no stream jump, bit 2 no 64-bit modulo; results then wrong) with the
# phase timestamps (PT_PART_PROF=1)
set -u
mkdir -p gpurun_out
T=${TAG:-r05an}
V=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
for dbg in 0 1 2 4 7; do
  PT_PART_PROF=1 PT_PART_DBG=$dbg timeout -k 10 300 python tools_gpu/ablib.py $V bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline --no-c3 --deterministic-timing 0 --repeats 1 > gpurun_out/${T}_dbg$dbg.log 2>&1 || exit $?
done
