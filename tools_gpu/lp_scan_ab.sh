#!/bin/bash
# The TransE link-prediction scan kernels (k_lp_scan_v, the default, vs k_lp_scan_t): the GPU tests that score
# link prediction, then C4 under rocprofv3 kernel statistics with each kernel (bench.py --lp-scan-kernel 0 | 1):
# scan time per launch and the rank digests of the two runs.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-lpab}
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread ${TESTS:-tests/test_gpu_lp_scan.py tests/test_gpu_pu.py tests/test_gpu_realscale.py} \
  -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
for k in 0 1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_k$k -o run --output-format csv -- \
    python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline --no-dropin --deterministic-timing 0 \
    --lp-scan-kernel $k > gpurun_out/${T}_c4_k$k.log 2>&1 || exit $?
done
