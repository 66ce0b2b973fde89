#!/bin/bash
# Round 5 (l): LP scan with its 8-dim groups unrolled by 2 vs without (same box), C4 kernel stats, then the GPU suite
set -u
mkdir -p gpurun_out
T=${TAG:-r05l}
R=openke-putranse_amd/openke/release
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-dropin --deterministic-timing 0"
for v in hip hip_prev; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_$v -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $R/libputranse_$v.so bench.py $A > gpurun_out/${T}_c4_$v.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_pytest.log 2>&1 || exit $?
