#!/bin/bash
# Round 4 (n): universe kernel variants on C3 (per-universe cycles): class 1 split by vector width (ab/lib_sv.so),
# one-negative steps linking their three entity rows at once (ab/lib_l3.so), each against the product.
set -u
mkdir -p gpurun_out
T=${TAG:-r04n}
# class 1 split by vector width (ab/lib_sv.so: scalar 5-8-float rows and float4 8-float rows in separate kernels)
for i in 1 2; do
  PT_UNI_PROF=1 timeout -k 10 300 python tools_gpu/ablib.py ab/lib_sv.so bench.py --workload c3 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_prof_sv_c3_$i.log 2>&1 || exit $?
  PT_UNI_PROF=1 timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_prof_prod_c3_$i.log 2>&1 || exit $?
done
# one-negative steps linking their three entity rows at once (ab/lib_l3.so) vs the product
TAG=${T}l LIBS="prod l3" WLS="c3 c4" bash tools_gpu/ab_libs.sh || exit $?
