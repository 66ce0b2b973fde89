#!/bin/bash
# Round 5 (g): GPU suite + drop-in host profile (C3) + drop-in legs C3 / C4 after the drop-in host changes
set -u
mkdir -p gpurun_out
T=${TAG:-r05g}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/prof_dropin.py c3 > gpurun_out/${T}_prof_c3.txt 2>&1 || exit $?
for w in c3 c4; do
  timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 \
    > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
