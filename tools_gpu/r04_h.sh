#!/bin/bash
# Round 4 (h): the C3 set's schedule (per-universe start / duration, PT_UNI_PROF dump), the default bench line
# (C2 + pu_c3 + the drop-in PU timing + CPU baselines), rocprofv3 kernel statistics of the driver-shaped C2 run.
set -u
mkdir -p gpurun_out
T=${TAG:-r04h}
PT_UNI_PROF=1 PT_UNI_PROF_DUMP=gpurun_out/${T}_prof_c3.npz timeout -k 10 300 python bench.py --workload c3 --steps 2 \
  --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c3prof.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${T}_default.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c2prof -o c2 -- python bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-dropin --repeats 1 --deterministic-timing 0 \
  > gpurun_out/${T}_c2prof.log 2>&1 || exit $?
# float4 TransE rows at 8 floats per lane (ab/lib_n4.so: PT_UNI_WIDE4=0, class-1 kernel, 1,024 threads) vs prod
TAG=${T}n LIBS="prod n4" WLS="c3 c4" bash tools_gpu/ab_libs.sh || exit $?
