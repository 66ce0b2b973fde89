#!/bin/bash
# Round 4 (o): each shape's universe run as a separate (non-inlined) function, so each is register-allocated alone
# (ab/lib_ni.so), against the product: per-universe cycles on C3, then C4 / C5 lines.
set -u
mkdir -p gpurun_out
T=${TAG:-r04o}
for i in 1 2; do
  PT_UNI_PROF=1 timeout -k 10 300 python tools_gpu/ablib.py ab/lib_ni.so bench.py --workload c3 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_ni_c3_$i.log 2>&1 || exit $?
  PT_UNI_PROF=1 timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_prod_c3_$i.log 2>&1 || exit $?
done
TAG=${T}w LIBS="prod ni" WLS="c4 c5" bash tools_gpu/ab_libs.sh || exit $?
