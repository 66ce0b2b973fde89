#!/bin/bash
# Round 5 (q): k_step_csr with the slot-scale mode's uncontracted v (product build) vs contracted (variant), same box
set -u
mkdir -p gpurun_out
T=${TAG:-r05q}
C="--no-cpu-baseline --no-c3 --deterministic-timing 0"
V=openke-putranse_amd/openke/release/libputranse_hip_vc.so
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $C > gpurun_out/${T}_prod_$i.log 2>&1 || exit $?
  timeout -k 10 300 python tools_gpu/ablib.py $V bench.py --steps 20 --warmup 5 $C > gpurun_out/${T}_vc_$i.log 2>&1 || exit $?
done
