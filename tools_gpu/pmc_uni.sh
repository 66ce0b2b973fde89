#!/bin/bash
# PMC passes over a universe workload (counters in separate passes, --kernel-trace only), summarised with the
# profiled library's sha256 into gpurun_out/pmc_<W>_uni.json.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=${W:-c3}
mkdir -p gpurun_out/pmcu_$W
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmcu_$W/p$i -o run --output-format csv -- python3 bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/pmcu_$W/p$i.log 2>&1 || exit $?
done
python3 tools_gpu/parse_pmc.py gpurun_out/pmcu_$W gpurun_out/pmc_${W}_uni.json > gpurun_out/pmcu_$W/summary.txt
