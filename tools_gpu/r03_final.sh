#!/bin/bash
# Round-3 closing evidence: GPU suite, smoke, driver-shaped and default bench lines, universe workloads,
# rocprofv3 kernel stats of the driver-shaped C2 run and of C3.
set -u
mkdir -p gpurun_out
T=${TAG:-r03f}
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_k20.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/${T}_k200.log 2>&1 || exit $?
for w in c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/${T}_prof20.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profc3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_profc3.log 2>&1 || exit $?
