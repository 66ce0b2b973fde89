#!/bin/bash
# Round 5 (m): the class-launch overlap test beside busy streams; rocprofv3 kernel statistics of the driver-shaped
# C2 command without the reference-order timing (only the fast path's kernels in the summary)
set -u
mkdir -p gpurun_out
T=${TAG:-r05m}
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_streams.py \
  > gpurun_out/${T}_pytest.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_k20 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --deterministic-timing 0 \
  > gpurun_out/${T}_prof_k20.log 2>&1 || exit $?
