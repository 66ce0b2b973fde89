#!/bin/bash
# SQ counters of the universe kernels on C3 (separate passes, --kernel-trace only).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcu
i=0
for set in "SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CU_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA" "SQ_INSTS_FLAT SQ_INSTS_SCRATCH SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmcu/p$i -o run --output-format csv -- python3 bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcu/p$i.log 2>&1
    rc=$?
    echo "pmc $i ($set) rc=$rc" >> gpurun_out/pmcu/steps.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python3 tools_gpu/parse_pmc.py gpurun_out/pmcu > gpurun_out/pmcu/summary.json
