#!/bin/bash
# Round 4 (p): hot single-shape universe kernels (product: the shapes of the set's longest universes in kernels
# compiled for that shape alone) vs the class kernels only (ab/lib_nohot.so): universe parity tests, then C3 / C4 / C5.
set -u
mkdir -p gpurun_out
T=${TAG:-r04p}
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py tests/test_gpu_ordered.py -m gpu > gpurun_out/${T}_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TAG=${T}a LIBS="prod nohot" WLS="c3 c4 c5" bash tools_gpu/ab_libs.sh || exit $?
