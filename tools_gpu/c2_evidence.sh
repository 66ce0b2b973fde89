#!/bin/bash
# C2 evidence on one GPU: default bench line, rocprofv3 kernel stats of the same command, PMC traffic.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
echo "bench rc=0" >> gpurun_out/steps.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/prof.log 2>&1 || exit $?
echo "prof rc=0" >> gpurun_out/steps.log
bash tools_gpu/pmc.sh c2 --no-c3 || exit $?
python3 tools_gpu/parse_pmc.py gpurun_out/pmc gpurun_out/pmc_c2.json > gpurun_out/pmc_summary.json 2>&1
