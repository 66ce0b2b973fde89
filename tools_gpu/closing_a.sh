#!/bin/bash
# Closing evidence A on the final build: the GPU suite with the forward-error log (PT_KAPPA_LOG), the chain counters
# of C4 / C3 / C5's longest universes (pmc_chain.sh), the driver's command and a rocprofv3 kernel-trace summary of it,
# then C2's PMC passes (pmc.sh). TAG names the outputs under gpurun_out/.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-closing}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 600 python -u -m pytest -q --timeout 200 \
  --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
python3 tools_gpu/kappa_summary.py gpurun_out/${T}_kappa.jsonl gpurun_out/${T}_parity_bound_summary.json \
  "PT_KAPPA_LOG of pytest -m gpu, final build" > gpurun_out/${T}_kappa_print.txt || exit $?
for w in c4 c3 c5; do W=$w TW=1 bash tools_gpu/pmc_chain.sh || exit $?; done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_default.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 \
  bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1 || exit $?
bash tools_gpu/pmc.sh || exit $?
