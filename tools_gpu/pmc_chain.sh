#!/bin/bash
# VALU / SALU / LDS / VMEM instruction counts of the longest universe of a workload trained alone in one workgroup
# (bench.py --longest-only --team-width 1), one --pmc pass with --kernel-trace; summarised with the library's sha256
# into gpurun_out/pmc_<W>_chain.json for bench.py's chain roofline (the VALU issue term of chain_floor).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=${W:-c4}
TW=${TW:-1}   # team width (1: the product's one-workgroup chain, which bench.py's roofline uses)
D=gpurun_out/pmcc_${W}_w$TW
mkdir -p $D
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $D/p1 -o run --output-format csv -- python3 bench.py \
  --workload $W --longest-only --team-width $TW --steps 1 --warmup 0 --no-cpu-baseline --no-dropin \
  --deterministic-timing 0 > $D/p1.log 2>&1 || exit $?
OUT=gpurun_out/pmc_${W}_chain.json
[ "$TW" = 1 ] || OUT=gpurun_out/pmc_${W}_chain_w$TW.json
python3 tools_gpu/parse_chain.py $D $OUT > $D/summary.txt
