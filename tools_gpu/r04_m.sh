#!/bin/bash
# Round 4 (m): the transposed link-prediction scan (k_lp_scan_t, product) vs the lane-group scan (ab/lib_ls0.so):
# the universe / LP parity tests on the product, then the C3 and C4 lines with their drop-in legs on both builds.
set -u
mkdir -p gpurun_out
T=${TAG:-r04m}
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in c3 c4; do
  timeout -k 10 400 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --deterministic-timing 0 \
    > gpurun_out/${T}_prod_$w.log 2>&1 || exit $?
  timeout -k 10 400 python tools_gpu/ablib.py ab/lib_ls0.so bench.py --workload $w --steps 1 --warmup 1 \
    --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_ls0_$w.log 2>&1 || exit $?
done
# the D 65-80 scalar-row shape alone in its class kernel (ab/lib_solo27.so: no other shape's registers; the
# other universes are NOT trained - a chain measurement only) vs the product, per-universe cycles
PT_UNI_PROF=1 timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
  --deterministic-timing 0 > gpurun_out/${T}_prof_prod_c3.log 2>&1 || exit $?
PT_UNI_PROF=1 timeout -k 10 300 python tools_gpu/ablib.py ab/lib_solo27.so bench.py --workload c3 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_prof_solo_c3.log 2>&1 || exit $?
