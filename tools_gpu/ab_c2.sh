#!/bin/bash
# Same-box A/B of product builds (LIBS) on the driver-shaped C2 command (--steps 20 --warmup 5), alternated;
# then the sampler parity tests on TESTLIB.
set -u
mkdir -p gpurun_out
T=${TAG:-abc2}
R=$PWD/openke-putranse_amd/openke/release
for rep in 1 2 3; do
  for l in ${LIBS:-base cand}; do
    PT_LIB_PATH=$R/libputranse_hip_$l.so timeout -k 10 200 python bench.py --steps ${K:-20} --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/${T}_${l}_$rep.log 2>&1 || exit $?
  done
done
if [ -n "${TESTLIB:-}" ]; then
  PT_LIB_PATH=$R/libputranse_hip_$TESTLIB.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sampling.py tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
fi
