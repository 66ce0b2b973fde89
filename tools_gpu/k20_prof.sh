#!/bin/bash
# Driver-shaped C2 bench (K=20, W=5) plus its rocprofv3 kernel stats, and the K=200 line for comparison.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/k20.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/k200.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/prof_k20.log 2>&1 || exit $?
