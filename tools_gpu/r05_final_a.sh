#!/bin/bash
# Round 5 closing evidence (a) on the final build: the whole GPU suite (forward-error bound log), smoke(), the
# default bench line, the driver-shaped C2 command, the C3 / C4 / C5 lines (drop-in legs, CPU baselines) and the
# rocprofv3 kernel statistics of the driver-shaped command.
set -u
mkdir -p gpurun_out
T=${TAG:-r05fa}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 300 python -u -m pytest -q --timeout 120 \
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
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_k20 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/${T}_prof_k20.log 2>&1 || exit $?
