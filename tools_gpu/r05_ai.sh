#!/bin/bash
# Round 5 (ai): TransH LP pairs two per pass (product build) vs one at a time (PT_LP_H2=0 build): the C5 line's
# drop-in (four validations over 256 PuTransH universes) twice each, kernel statistics of one; TransH LP tests first
set -u
mkdir -p gpurun_out
T=${TAG:-r05ai}
R=openke-putranse_amd/openke/release
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pu.py \
  tests/test_gpu_configs.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--workload c5 --steps 1 --warmup 0 --no-cpu-baseline --deterministic-timing 0"
for v in hip hip_h1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c5_$v -o run --output-format csv -- \
    python3 tools_gpu/ablib.py $R/libputranse_$v.so bench.py $A > gpurun_out/${T}_c5_${v}_1.log 2>&1 || exit $?
  timeout -k 10 300 python tools_gpu/ablib.py $R/libputranse_$v.so bench.py $A > gpurun_out/${T}_c5_${v}_2.log 2>&1 || exit $?
done
