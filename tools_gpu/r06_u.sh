#!/bin/bash
# Round 6 (u): TransH float4 rows at one chunk per lane in a hot 1,024-thread kernel - the universe tests (TransH
# universes teacher-forced against the oracle, C5's config test, the reference-order kernels), then same-box A/B of
# C5 against the build with two chunks per lane (PT_UNI_TRANSH_F4=2).
set -u
mkdir -p gpurun_out
T=${TAG:-r06u}
TH2=openke-putranse_amd/openke/release/libputranse_hip_th2.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py tests/test_gpu_ordered.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 300 python tools_gpu/ablib.py $TH2 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c5_th2_$k.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_c5_new_$k.log 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --workload c5 --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline --no-dropin \
  --deterministic-timing 0 > gpurun_out/${T}_c5_p8.log 2>&1 || exit $?
