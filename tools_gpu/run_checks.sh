#!/bin/bash
# GPU-box check script: tests, smoke, bench, profile. Stops at the first fault/abort/timeout.
set -u
mkdir -p gpurun_out
step() {  # name, timeout, command...
    local name=$1 to=$2; shift 2
    echo "== $name" >> gpurun_out/steps.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" >> gpurun_out/steps.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >> gpurun_out/steps.log; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
    step gpu_tests 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = smoke ]; then
    step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 400 python bench.py --steps 100 --warmup 10 --cpu-seconds 10
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
    step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline
fi
exit 0
