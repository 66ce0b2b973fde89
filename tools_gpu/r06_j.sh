#!/bin/bash
# Round 6 (j): private-L2 universes - the universe tests, then C4 / C3 / C5 and the C4 / C3 8-way shares with
# isolation (library default) and without (--isolation 0).
set -u
mkdir -p gpurun_out
T=${TAG:-r06j}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py -m gpu \
  > gpurun_out/${T}_pu_tests.log 2>&1 || exit $?
for w in c4 c3 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
    --deterministic-timing 0 > gpurun_out/${T}_${w}.log 2>&1 || exit $?
done
for w in c4 c3; do
  for iso in 7 0; do
    timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --place-world 8 --isolation $iso \
      --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_${w}_p8_i$iso.log 2>&1 || exit $?
  done
done
