#!/bin/bash
# Round 5 (ae): a positive's three universe sink calls batched (UniverseSink::pos3, product build) vs one by one
# (PT_UNI_POS3=0 build), same box, interleaved: C3 / C4 lines; then the universe parity tests on the product build
set -u
mkdir -p gpurun_out
T=${TAG:-r05ae}
R=openke-putranse_amd/openke/release
A="--steps 3 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_modes.py tests/test_gpu_streams.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
for i in 1 2; do
  for v in hip hip_p3off; do
    for w in c3 c4; do
      timeout -k 10 300 python tools_gpu/ablib.py $R/libputranse_$v.so bench.py --workload $w $A > gpurun_out/${T}_${v}_${w}_$i.log 2>&1 || exit $?
    done
  done
done
