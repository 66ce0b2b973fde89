#!/bin/bash
# Round 5 (p): slot-scale mode (per-slot records + positive base rows instead of contribution rows) - its GPU test
# and the suite, then the C2 lines with it off / on (alternating, same box) and rocprofv3 statistics of both
set -u
mkdir -p gpurun_out
T=${TAG:-r05p}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_pytest.log 2>&1 || exit $?
C="--no-cpu-baseline --no-c3 --deterministic-timing 0"
for i in 1 2; do
  for m in 0 1; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --slot-scale $m $C > gpurun_out/${T}_k20_sc${m}_$i.log 2>&1 || exit $?
    timeout -k 10 300 python bench.py --slot-scale $m $C > gpurun_out/${T}_k200_sc${m}_$i.log 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_sc$m -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --slot-scale $m $C > gpurun_out/${T}_prof_sc$m.log 2>&1 || exit $?
done
