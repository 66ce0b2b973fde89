#!/bin/bash
# Same-box A/B of two library builds (ab/lib_old.so vs the tree's) on C3 / C4 / C5, interleaved.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for w in c3 c4 c5; do
    PT_LIB_PATH=$GRAFT_REPO_ROOT/ab/lib_old.so timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_old_${w}_$rep.log 2>&1 || exit $?
    timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_new_${w}_$rep.log 2>&1 || exit $?
  done
done
