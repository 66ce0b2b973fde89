#!/bin/bash
# Round 5 (c): kernel traces of the default bench process (round 4's per-set side streams vs the product's
# dedicated-queue class streams: Queue_Id and start / end of the four k_universes launches); the reference
# experiment's own scale (experiments/static_experiment_PuTransE_on_WN18.py: 6,000 universes, dim 20, valid_steps
# 100, then run_link_prediction) as kernel-only and drop-in lines; 8-way placement shares of C4, C5 and a 4,096-
# universe C3 wave.
set -u
mkdir -p gpurun_out
T=${TAG:-r05c}
TL=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
COMMON="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --deterministic-timing 0"
timeout -k 10 900 python bench.py --workload c3 --universes 6000 --dim 20 --valid-steps 100 --link-prediction \
  --steps 2 --warmup 1 --deterministic-timing 0 > gpurun_out/${T}_c3_6000.log 2>&1 || exit $?
for w in c4 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --place-world 8 \
    --deterministic-timing 0 > gpurun_out/${T}_${w}_place8.log 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --workload c3 --universes 4096 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
  --place-world 8 --deterministic-timing 0 > gpurun_out/${T}_c3w4096_place8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace_prod -o run --output-format csv -- \
  python3 bench.py $COMMON > gpurun_out/${T}_trace_prod.log 2>&1 || exit $?
PT_UNI_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace_tun0 -o run \
  --output-format csv -- python3 tools_gpu/ablib.py $TL bench.py $COMMON > gpurun_out/${T}_trace_tun0.log 2>&1 || exit $?
