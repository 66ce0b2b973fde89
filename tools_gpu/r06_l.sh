#!/bin/bash
# Round 6 (l): C4's 8-way shares with private-L2 universes: which universes end each share, and on which XCDs.
set -u
mkdir -p gpurun_out
T=${TAG:-r06l}
timeout -k 10 400 python bench.py --workload c4 --steps 1 --warmup 1 --place-world 8 --no-cpu-baseline --no-dropin \
  --deterministic-timing 0 > gpurun_out/${T}_c4_p8.log 2>&1 || exit $?
