#!/bin/bash
# Round 5 (u): split sampling of the driver's 20-step chunk. GPU sampling tests; then the driver's command with
# the tuning build at PT_SAMPLE_SPLIT = 0 (one launch) / 1 / 2 / 4, interleaved; a kernel trace of the default
set -u
mkdir -p gpurun_out
T=${TAG:-r05u}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampling.py \
  > gpurun_out/${T}_tests.log 2>&1 || exit $?
V=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
C="--steps 20 --warmup 5 --no-cpu-baseline --no-c3 --deterministic-timing 0"
for i in 1 2 3; do
  for h in 0 1 2 4; do
    PT_SAMPLE_SPLIT=$h timeout -k 10 300 python tools_gpu/ablib.py $V bench.py $C > gpurun_out/${T}_h${h}_$i.log 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run -- python bench.py $C \
  > gpurun_out/${T}_trace.log 2>&1 || exit $?
