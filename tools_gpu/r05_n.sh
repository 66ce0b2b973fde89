#!/bin/bash
# Round 5 (n): the overlap test under round 4's stream scheme (tuning build, PT_UNI_STREAMS=0) must FAIL - the
# test detects the serialization it guards against
set -u
mkdir -p gpurun_out
T=${TAG:-r05n}
PT_UNI_STREAMS=0 timeout -k 10 200 python tools_gpu/ablib.py openke-putranse_amd/openke/release/libputranse_hip_tuning.so \
  -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py > gpurun_out/${T}_pytest.log 2>&1; echo "rc=$?" >> gpurun_out/${T}_pytest.log; timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py > gpurun_out/${T}_pytest_prod.log 2>&1
echo "rc=$?" >> gpurun_out/${T}_pytest.log
