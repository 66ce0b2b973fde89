#!/bin/bash
# Round 6 (q), evidence B: C2's counted traffic (pmc.sh, the driver-shaped command), the C4 / C3 / C5 lines with
# their 8-way shares and drop-in legs (chain roofline with the committed VALU counts), the N = 2 rehearsal over gloo
# (pu_c4_lp digest), and smoke().
set -u
mkdir -p gpurun_out
T=${TAG:-r06q}
bash tools_gpu/pmc.sh || exit $?
for w in c4 c3 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --no-cpu-baseline \
    > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
PT_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/${T}_dist2.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 \
  || exit $?
