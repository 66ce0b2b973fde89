#!/bin/bash
# Round evidence on one GPU: GPU tests, smoke, default bench (C2 + pu_c3 + CPU baseline), rocprofv3 kernel
# stats of the C2 bench and of C3, C3/C4/C5 bench lines. Stops at the first failure.
set -u
mkdir -p gpurun_out
echo "start" > gpurun_out/steps.log
step() {  # name, timeout, command...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" >> gpurun_out/steps.log
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step gpu_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
for wl in c3 c4 c5; do step bench_$wl 400 python bench.py --workload $wl --steps 2 --warmup 1 --cpu-seconds 10; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-c3
step prof_c3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
bash tools_gpu/pmc.sh c2 --no-c3 || exit $?
python3 tools_gpu/parse_pmc.py gpurun_out/pmc gpurun_out/pmc_c2.json > gpurun_out/pmc_summary.json 2>&1
echo "pmc done" >> gpurun_out/steps.log
