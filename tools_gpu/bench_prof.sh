#!/bin/bash
# default bench line + rocprofv3 kernel stats of the same kind of run
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-c3 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-c3 > gpurun_out/prof.log 2>&1 || exit $?
