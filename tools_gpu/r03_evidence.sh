#!/bin/bash
# Round-3 evidence: GPU suite, smoke, default bench line, universe workloads, rocprofv3 stats of the bench
set -u
mkdir -p gpurun_out
T=${TAG:-r03e}
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
for w in c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-c3 > gpurun_out/${T}_prof.log 2>&1 || exit $?
