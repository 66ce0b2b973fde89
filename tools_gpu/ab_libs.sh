#!/bin/bash
# Same-box A/B over several builds of the library (ab/lib_<name>.so; the name "prod" = the product library
# openke/release/libputranse_hip.so), alternated on the universe workloads (WLS) with phase profiling; then
# the universe parity tests on TESTLIB. Alternative builds load through tools_gpu/ablib.py (the product
# loader reads no environment variable).
set -u
mkdir -p gpurun_out
T=${TAG:-ab}
libpath() { if [ "$1" = prod ]; then echo openke-putranse_amd/openke/release/libputranse_hip.so; else echo ab/lib_$1.so; fi; }
for rep in 1 2; do
  for w in ${WLS:-c3 c4 c5}; do
    for l in ${LIBS:-base prod}; do
      PT_UNI_PROF=1 timeout -k 10 200 python tools_gpu/ablib.py $(libpath $l) bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/${T}_${l}_${w}_$rep.log 2>&1 || exit $?
    done
  done
done
if [ -n "${TESTLIB:-}" ]; then
  timeout -k 10 600 python -u tools_gpu/ablib.py $(libpath $TESTLIB) -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
fi
