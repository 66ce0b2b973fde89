#!/bin/bash
# Round 4 closing evidence (a) on the final build: the whole GPU suite (forward-error bound log), smoke(), the
# default bench line (C2 200-step epochs + pu_c3 + its drop-in leg + CPU baselines), the driver-shaped C2
# command, the C3 / C4 / C5 lines (drop-in legs for C3 and C4) and the 8-way placement shares of C3.
set -u
mkdir -p gpurun_out
T=${TAG:-r04fa}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 900 python -u -m pytest -q --timeout 300 \
  --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 \
  || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${T}_default.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_driver.log 2>&1 || exit $?
for w in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 > gpurun_out/${T}_$w.log 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --place-world 8 \
  --deterministic-timing 0 > gpurun_out/${T}_place8.log 2>&1 || exit $?
# the N > 1 bench path rehearsed on this one-GPU box: 2 ranks over gloo sharing the GPU
bash tools_gpu/dist_rehearsal.sh || exit $?
