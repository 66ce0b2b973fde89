#!/bin/bash
# apply-kernel variants, universe relation-list path, GPU parity tests.
set -u
mkdir -p gpurun_out
for v in "PT_APPLY_RPW=1" "PT_APPLY_RPW=2" "PT_APPLY_RPW=4"; do
    echo "== $v" >> gpurun_out/c2_ab.log
    env $v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 >> gpurun_out/c2_ab.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc" >> gpurun_out/c2_ab.log; exit $rc; fi
done
for v in "PT_UNI_RELGRAD=1" "PT_UNI_RELGRAD=0"; do
    echo "== $v" >> gpurun_out/c2_ab.log
    env $v timeout -k 10 200 python bench.py --workload c3 --steps 2 --warmup 1 >> gpurun_out/c2_ab.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc" >> gpurun_out/c2_ab.log; exit $rc; fi
done
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit $?
PT_UNI_RELGRAD=0 timeout -k 10 300 python -m pytest tests/test_gpu_pu.py -q -x -p no:cacheprovider > gpurun_out/pu_tests_rellist.log 2>&1
