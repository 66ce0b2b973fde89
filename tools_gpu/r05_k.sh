#!/bin/bash
# Round 5 (k): LP scan with scalar (uniform) pair walk and prefetched key-row cells - GPU suite + C4 kernel stats
set -u
mkdir -p gpurun_out
T=${TAG:-r05k}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_pytest.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4 -o run --output-format csv -- \
  python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
  > gpurun_out/${T}_c4.log 2>&1 || exit $?
