#!/bin/bash
# Split sampler (k_sample_part): batch parity tests, then C2 bench lines per sampling path at K=20 / K=200
# and a rocprofv3 kernel-stats run of the driver-shaped K=20 line.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sampling.py \
    tests/test_gpu_parity.py -k "sampling or fused" > gpurun_out/pytest_sampling.log 2>&1 || exit $?
for mode in auto part twopass fused; do
  for k in 20 200; do
    w=$(( k / 4 )); [ $w -lt 5 ] && w=5
    if [ $mode = auto ]; then
      timeout -k 10 200 python bench.py --steps $k --warmup $w --no-cpu-baseline --no-c3 > gpurun_out/ab_${mode}_k$k.log 2>&1 || exit $?
    else
      PT_SAMPLE_MODE=$mode timeout -k 10 200 python bench.py --steps $k --warmup $w --no-cpu-baseline --no-c3 > gpurun_out/ab_${mode}_k$k.log 2>&1 || exit $?
    fi
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_part_k20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/prof_part_k20.log 2>&1 || exit $?
