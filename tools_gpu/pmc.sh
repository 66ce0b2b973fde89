#!/bin/bash
# PMC passes over the driver-shaped C2 bench run (counters collected in separate passes, --kernel-trace only),
# summarised into gpurun_out/pmc_c2.json with the profiled library's sha256 (bench.py reads it from profiles/
# only when the digest matches the library it loaded).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
K=${STEPS:-20}; W=${WARMUP:-5}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py --steps $K --warmup $W --repeats 1 --deterministic-timing 0 --no-cpu-baseline --no-c3 > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done
# sampled steps of that command: warmup W + graph capture K + timed K + the per-kernel timing run K
python3 tools_gpu/parse_pmc.py gpurun_out/pmc gpurun_out/pmc_c2.json $((W + 3 * K)) > gpurun_out/pmc/summary.txt
