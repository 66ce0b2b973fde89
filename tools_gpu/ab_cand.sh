#!/bin/bash
# Same-box A/B: A = a baseline product build (libputranse_hip_base.so), B = a candidate product build
# (libputranse_hip_cand.so, a candidate change), alternated on the universe workloads with phase
# profiling; then the universe parity tests on B.
set -u
mkdir -p gpurun_out
T=${TAG:-ab}
R=$PWD/openke-putranse_amd/openke/release
for rep in 1 2; do
  for w in ${WLS:-c3 c4 c5}; do
    PT_UNI_PROF=1 PT_LIB_PATH=$R/libputranse_hip_base.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_A_${w}_$rep.log 2>&1 || exit $?
    PT_UNI_PROF=1 PT_LIB_PATH=$R/libputranse_hip_cand.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_B_${w}_$rep.log 2>&1 || exit $?
  done
done
PT_LIB_PATH=$R/libputranse_hip_cand.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
