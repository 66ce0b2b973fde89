#!/bin/bash
# Round 5 (e): GPU-drawn initial universe tables - the GPU suite (incl. test_gpu_init.py), then the drop-in
# legs of C3 (512 universes) and of the reference experiment's scale (6,000 universes, dim 20, valid_steps 100).
set -u
mkdir -p gpurun_out
T=${TAG:-r05e}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 \
  > gpurun_out/${T}_c3.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c3 --universes 6000 --dim 20 --valid-steps 100 --link-prediction \
  --steps 2 --warmup 1 --no-cpu-baseline --deterministic-timing 0 > gpurun_out/${T}_c3_6000.log 2>&1 || exit $?
