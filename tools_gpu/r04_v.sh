#!/bin/bash
# Round 4 (v): CU shares from a fixed + per-positive step-cost model (product) against the fixed + rounds model
# (ab/lib_old.so): C3 / C4 / C5 alternated with per-universe schedules, then the universe parity tests on the product,
# then C3's 8-way placement shares on the product.
set -u
TAG=r04v LIBS="old prod" WLS="c3 c5" STEPS=3 TESTLIB=prod bash tools_gpu/ab_libs.sh || exit $?
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
  --place-world 8 > gpurun_out/r04v_place8.log 2>&1 || exit $?
