#!/bin/bash
# Round 5: the universe trainer's class launches in a process that already holds streams (the default bench line:
# C2 trainer + capture stream, then the C3 set) against the standalone C3 line. Product build (full-CU-mask class
# streams) and the tuning build's PT_UNI_STREAMS = 0 (round 4's per-set side streams), 2 (high priority), 3 (plain
# library streams). Each line carries pu_c3.class_launches (per launch start / end, overlap).
set -u
mkdir -p gpurun_out
T=${TAG:-r05a}
TL=openke-putranse_amd/openke/release/libputranse_hip_tuning.so
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log; [ $rc -le 1 ] || exit $rc
COMMON="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --deterministic-timing 0"
timeout -k 10 300 python bench.py $COMMON > gpurun_out/${T}_default_prod.log 2>&1 || exit $?
for m in 0 2 3 1; do
  PT_UNI_STREAMS=$m timeout -k 10 300 python tools_gpu/ablib.py $TL bench.py $COMMON \
    > gpurun_out/${T}_default_tun$m.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
  --deterministic-timing 0 > gpurun_out/${T}_c3_prod.log 2>&1 || exit $?
PT_UNI_STREAMS=0 timeout -k 10 300 python tools_gpu/ablib.py $TL bench.py --workload c3 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c3_tun0.log 2>&1 || exit $?
