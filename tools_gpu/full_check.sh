#!/bin/bash
# Full GPU evidence: tests, smoke, C2 bench + rocprof, then C3/C4/C5 bench lines. Stops at the first failure.
set -u
mkdir -p gpurun_out
bash tools_gpu/run_checks.sh all || exit $?
for wl in c3 c4 c5; do
    echo "== bench_$wl" >> gpurun_out/steps.log
    timeout -k 10 400 python bench.py --workload $wl --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_$wl.log 2>&1 || exit $?
    echo "bench_$wl rc=0" >> gpurun_out/steps.log
done
exit 0
