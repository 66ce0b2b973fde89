#!/bin/bash
# Round 4 (c): A/B of the universe kernel builds - prod (shape classes 5-6 / 7-8 floats split, joint
# normalization for <= 6 floats, 1,024 threads for TransE classes 0-2), c2 (the 7-8 class at 512 threads),
# u1024 (one 5-8 class at 1,024 threads, no joint reductions), g0 (flat masked row access) - then per-universe
# phase profiles (dumps for the CU-share time model) and the placement shares of C3. A GPU fault / timeout
# ends the script.
set -u
mkdir -p gpurun_out
T=${TAG:-r04c}
TAG=${T}a LIBS="prod c2 u1024" WLS="c3" bash tools_gpu/ab_libs.sh || exit $?
TAG=${T}b LIBS="prod u1024 g0" WLS="c4 c5" bash tools_gpu/ab_libs.sh || exit $?
for w in c3 c4 c5; do
  PT_UNI_PROF=1 PT_UNI_PROF_DUMP=gpurun_out/${T}_prof_$w.npz timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --place-world 8 > gpurun_out/${T}_place8.log 2>&1 || exit $?
