#!/bin/bash
# Round 5 (i): the transposed LP scan scoring two pairs per pass over the LDS row - GPU suite, then rocprofv3 kernel
# statistics of C4 (link prediction over 1,024 universes) for this build and the previous one (same box).
set -u
mkdir -p gpurun_out
T=${TAG:-r05i}
P=openke-putranse_amd/openke/release/libputranse_hip_prev.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_pytest.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_new -o run --output-format csv -- \
  python3 bench.py $A > gpurun_out/${T}_c4_new.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_prev -o run --output-format csv -- \
  python3 tools_gpu/ablib.py $P bench.py $A > gpurun_out/${T}_c4_prev.log 2>&1 || exit $?
