#!/bin/bash
# Round 4 closing evidence (b) on the final build: rocprofv3 kernel statistics of the driver-shaped C2 command and of
# the C3 line, then the PMC counter passes (C2: tools_gpu/pmc.sh -> gpurun_out/pmc_c2.json; C3 universes:
# tools_gpu/pmc_uni.sh -> gpurun_out/pmc_c3_uni.json), each stamped with the profiled library's sha256.
set -u
mkdir -p gpurun_out
T=${TAG:-r04fb}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c2 -o run -- python bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin --repeats 1 --deterministic-timing 0 \
  > gpurun_out/${T}_c2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3 -o run -- python bench.py \
  --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
  > gpurun_out/${T}_c3.log 2>&1 || exit $?
bash tools_gpu/pmc.sh || exit $?
W=c3 bash tools_gpu/pmc_uni.sh || exit $?
