#!/bin/bash
# Round 5 (o): phase timestamps of the split sampler (k_sample_part) on the driver-shaped C2 command (tuning build)
set -u
mkdir -p gpurun_out
T=${TAG:-r05o}
PT_PART_PROF=1 timeout -k 10 300 python tools_gpu/ablib.py openke-putranse_amd/openke/release/libputranse_hip_tuning.so \
  bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --deterministic-timing 0 > gpurun_out/${T}_k20.log 2>&1 || exit $?
