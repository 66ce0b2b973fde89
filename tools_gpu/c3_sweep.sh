#!/bin/bash
# C3 (PuTransE universes) run with per-phase profile, then without.
set -u
mkdir -p gpurun_out
for cfg in "1" "0"; do
    set -- $cfg
    echo "== prof=$1" >> gpurun_out/c3_sweep.log
    PT_UNI_PROF=$1 timeout -k 10 120 python bench.py --workload c3 --steps 2 --warmup 1 >> gpurun_out/c3_sweep.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc" >> gpurun_out/c3_sweep.log; exit $rc; fi
done
