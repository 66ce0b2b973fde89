#!/bin/bash
# Round 6 (r), evidence C: the driver's command (C2 with counted traffic now that pmc_c2.json is this build's), the
# C4 / C3 / C5 lines with 8-way shares and drop-in legs (chain roofline with the committed VALU counts), and a
# rocprofv3 kernel-trace summary of each universe line.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r06r}
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_default.log 2>&1 || exit $?
for w in c4 c3 c5; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
    > gpurun_out/${T}_$w.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_${w}_prof -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    > gpurun_out/${T}_${w}_prof.log 2>&1 || exit $?
done
