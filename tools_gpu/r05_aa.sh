#!/bin/bash
# Round 5 (aa): is k_step_csr slower after the split sampler (rank_only: the step adds start[e]) or at K = 20?
# Tuning build, sampling path forced: fused / part at K = 20 and K = 200, twice each
set -u
mkdir -p gpurun_out
T=${TAG:-r05aa}
V=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
for i in 1 2; do
  for m in fused part; do
    for k in 20 200; do
      PT_SAMPLE_MODE=$m timeout -k 10 300 python tools_gpu/ablib.py $V bench.py --steps $k --warmup 5 --no-cpu-baseline \
        --no-c3 --deterministic-timing 0 --repeats 3 > gpurun_out/${T}_${m}_k${k}_$i.log 2>&1 || exit $?
    done
  done
done
