#!/bin/bash
# Round 5 closing evidence (b): rocprofv3 --pmc passes of the driver-shaped C2 command (pmc.sh -> pmc_c2.json,
# stamped with the library's sha256), the default line re-run so its roofline carries the counted traffic of this
# build, rocprofv3 kernel statistics of the C3 / C5 lines, the reference experiment's 6,000 universes, and the N = 2
# rehearsal over gloo on this one GPU.
set -u
mkdir -p gpurun_out
T=${TAG:-r05fb}
bash tools_gpu/pmc.sh || exit $?
cp gpurun_out/pmc_c2.json profiles/pmc_c2.json || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${T}_default_counted.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$w -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
    > gpurun_out/${T}_prof_$w.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py --workload c3 --universes 6000 --dim 20 --valid-steps 100 --link-prediction \
  --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_c3_6000.log 2>&1 || exit $?
bash tools_gpu/dist_rehearsal.sh || exit $?
