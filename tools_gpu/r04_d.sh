#!/bin/bash
# Round 4 (d): the fused step + apply (C2) - its parity tests, then the driver-shaped C2 line fused vs the
# step + apply pair (alternated), a rocprofv3 kernel summary of the fused C2 run; universe builds A/B:
# prod (shape classes 5-6 / 7-8 split, HBM-typed rows up to 8 floats per lane), ns (one 5-8 class), gf (flat
# rows everywhere). A GPU fault / timeout ends the script; a test failure does not skip the measurements.
set -u
mkdir -p gpurun_out
T=${TAG:-r04d}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "step_apply or counting_sort or full_size or teacher_forced" -m gpu > gpurun_out/${T}_fused_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_fused_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  for sa in 1 0; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin --step-apply $sa \
      > gpurun_out/${T}_c2_sa${sa}_$i.log 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o c2 -- python bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-c3 --no-dropin --repeats 1 --deterministic-timing 0 > gpurun_out/${T}_c2_prof.log 2>&1 || exit $?
TAG=${T}u LIBS="prod ns gf" WLS="c3" bash tools_gpu/ab_libs.sh || exit $?
TAG=${T}v LIBS="prod gf" WLS="c5 c4" bash tools_gpu/ab_libs.sh || exit $?
