#!/bin/bash
# Same-box A/B over several product builds (openke/release/libputranse_hip_<name>.so, LIBS="base cand1 ..."),
# alternated on the universe workloads (WLS) with phase profiling; then the universe parity tests on TESTLIB.
set -u
mkdir -p gpurun_out
T=${TAG:-ab}
R=$PWD/openke-putranse_amd/openke/release
for rep in 1 2; do
  for w in ${WLS:-c3 c4 c5}; do
    for l in ${LIBS:-base cand}; do
      PT_UNI_PROF=1 PT_LIB_PATH=$R/libputranse_hip_$l.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${l}_${w}_$rep.log 2>&1 || exit $?
    done
  done
done
if [ -n "${TESTLIB:-}" ]; then
  PT_LIB_PATH=$R/libputranse_hip_$TESTLIB.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
fi
