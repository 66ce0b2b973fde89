#!/bin/bash
# universe kernel cycle split (PT_UNI_PROF=1) for C3 and C5 ($UNI_ENV: extra env for C3 variants, ';'-separated)
set -u
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${UNI_ENV:-PT_DUMMY=0}"
for v in "${VS[@]}"; do
    echo "== c3 $v" >> gpurun_out/uni_prof.log
    env $v PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/uni_prof.log 2>&1 || exit $?
done
echo "== c5" >> gpurun_out/uni_prof.log
PT_UNI_PROF=1 timeout -k 10 200 python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/uni_prof.log 2>&1 || exit $?
