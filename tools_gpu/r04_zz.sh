#!/bin/bash
# Round 4 (zz): on the final build, the whole -m gpu suite once more (a second box) and rocprofv3 kernel statistics of
# the C4 and C5 lines (the C2 and C3 ones are r04_final_b.sh's).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r04zz_pytest.log 2>&1 \
  || exit $?
for w in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04zz_$w -o run -- python bench.py \
    --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/r04zz_$w.log 2>&1 \
    || exit $?
done
