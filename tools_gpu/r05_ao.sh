#!/bin/bash
# Round 5 (ao): the split sampler's slot draws by fastmod reciprocals precomputed per positive (product build) vs
# the 64-bit `%` (the previous commit's build), same box, interleaved on the driver's command; sampling and
# C2 parity tests on the product build first; the phase profile of the tuning build
set -u
mkdir -p gpurun_out
T=${TAG:-r05ao}
R=openke-putranse_amd/openke/release
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampling.py \
  tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
C="--steps 20 --warmup 5 --no-cpu-baseline --no-c3 --deterministic-timing 0 --repeats 3"
for i in 1 2 3; do
  for v in hip hip_prev; do
    timeout -k 10 300 python tools_gpu/ablib.py $R/libputranse_$v.so bench.py $C > gpurun_out/${T}_${v}_$i.log 2>&1 || exit $?
  done
done
PT_PART_PROF=1 timeout -k 10 300 python tools_gpu/ablib.py $R/libputranse_hip_tuning.so bench.py $C --repeats 1 \
  > gpurun_out/${T}_prof.log 2>&1 || exit $?
