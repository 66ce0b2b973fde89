#!/bin/bash
# Round 4: the whole GPU suite with the forward-error (kappa) bound log; a test failure does not hide the log
set -u
mkdir -p gpurun_out
T=${TAG:-r04t}
PT_KAPPA_LOG=$PWD/gpurun_out/${T}_kappa.jsonl timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
exit $rc
