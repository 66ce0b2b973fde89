#!/bin/bash
# Round-end evidence on one GPU: GPU tests, smoke, default bench, C3 bench, rocprofv3 kernel stats, PMC.
set -u
mkdir -p gpurun_out
bash tools_gpu/run_checks.sh all || exit $?
timeout -k 10 200 python bench.py --workload c3 --steps 3 --warmup 1 > gpurun_out/bench_c3.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 2 --warmup 1 > gpurun_out/prof_c3.log 2>&1 || exit $?
bash tools_gpu/pmc.sh c2 || exit $?
python3 tools_gpu/parse_pmc.py gpurun_out/pmc gpurun_out/pmc_c2.json > gpurun_out/pmc_summary.json 2>&1
