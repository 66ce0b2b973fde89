#!/bin/bash
# Round 4 (t): LCG stream jumps from a constant table of the maps LCG^(2^i) (ab/lib_tj.so) against the product:
# the whole -m gpu suite on ab/lib_tj.so (the samplers are bit-exact against the oracle), then the driver-shaped C2
# command and the universe workloads, alternated; ab/lib_rt.so = lib_tj plus the relation rows found by a flag
# scan in phase B (PT_UNI_RELSCAN) instead of returning LDS atomics in phase A.
set -u
mkdir -p gpurun_out
T=r04t
P=openke-putranse_amd/openke/release/libputranse_hip.so
timeout -k 10 600 python -u tools_gpu/ablib.py ab/lib_tj.so -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_tests.log 2>&1 || exit $?
for rep in 1 2; do
  for l in prod tj rt; do
    lp=$P; [ $l != prod ] && lp=ab/lib_$l.so
    timeout -k 10 200 python tools_gpu/ablib.py $lp bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin \
      --deterministic-timing 0 > gpurun_out/${T}_${l}_c2_$rep.log 2>&1 || exit $?
  done
done
TAG=$T LIBS="prod tj rt" WLS="c3 c4 c5" STEPS=3 bash tools_gpu/ab_libs.sh
