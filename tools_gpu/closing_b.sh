#!/bin/bash
# Closing evidence B on the final build (after closing_a.sh's pmc_c2.json and pmc_c*_chain.json are committed under
# profiles/): the driver's command with counted traffic, the C4 / C3 / C5 lines with 8-way shares and drop-in legs
# and their kernel stats, the reference experiment's scale, the N = 2 gloo rehearsal and smoke().
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-closingb}
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_default.log 2>&1 || exit $?
for w in c4 c3 c5; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
    > gpurun_out/${T}_$w.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_${w}_prof -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
    > gpurun_out/${T}_${w}_prof.log 2>&1 || exit $?
done
timeout -k 10 400 python3 bench.py --workload c3 --universes 6000 --dim 20 --valid-steps 100 --link-prediction \
  --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_ref6000.log 2>&1 || exit $?
PT_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/${T}_dist2.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 \
  || exit $?
