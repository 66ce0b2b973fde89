#!/bin/bash
# Extra SQ counters on the C2 step (separate passes, --kernel-trace only).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcx
i=0
for set in "SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CU_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmcx/p$i -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 > gpurun_out/pmcx/p$i.log 2>&1
    rc=$?
    echo "pmc $i ($set) rc=$rc" >> gpurun_out/pmcx/steps.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python3 tools_gpu/parse_pmc.py gpurun_out/pmcx > gpurun_out/pmcx/summary.json
