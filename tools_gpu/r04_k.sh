#!/bin/bash
# Round 4 (k): kernel statistics of the C3 workload line with its drop-in leg (universe kernels, the link-
# prediction fold kernels of the 4 validations, ranking) and of the C4 line (drop-in + run_link_prediction).
set -u
mkdir -p gpurun_out
T=${TAG:-r04k}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in c3 c4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_$w -o run -- python bench.py \
    --workload $w --steps 1 --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
