#!/bin/bash
# Round-2 closing evidence on one GPU: GPU tests, smoke, the driver-shaped default bench line (K=20, W=5),
# the K=200 line, rocprofv3 kernel stats of the driver-shaped command, and the C3 / C4 / C5 universe lines.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/ev_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ev_bench_k20.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/ev_bench_k200.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_prof_k20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ev_prof_k20.log 2>&1 || exit $?
for w in c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 > gpurun_out/ev_bench_$w.log 2>&1 || exit $?
done
