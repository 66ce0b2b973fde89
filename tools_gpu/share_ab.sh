#!/bin/bash
# Universe CU placement A/B (tuning build, host-side knobs only): the default CU-share model, the model
# with a larger fixed per-step cost (PT_UNI_FIXED), and one workgroup per universe (PT_UNI_GRID=1).
set -u
mkdir -p gpurun_out
T=${TAG:-sh}
export PT_LIB_PATH=$PWD/openke-putranse_amd/openke/release/libputranse_hip_tuning.so
for w in ${WLS:-c3 c4 c5}; do
  for arm in "def" "PT_UNI_FIXED=4" "PT_UNI_FIXED=8" "PT_UNI_GRID=1"; do
    tag=$(echo $arm | tr '=' '_')
    if [ "$arm" = def ]; then
      timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${tag}_$w.log 2>&1 || exit $?
    else
      env $arm timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${tag}_$w.log 2>&1 || exit $?
    fi
  done
done
