#!/bin/bash
# full GPU suite, smoke, default bench line
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r03_mid_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_mid_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r03_mid_bench.log 2>&1 || exit $?
