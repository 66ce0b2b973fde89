#!/bin/bash
# N > 1 rehearsal of bench.py on a one-GPU box: 2 ranks over gloo sharing the GPU (the driver runs N ranks
# over RCCL, one per GPU). Checks the multi-rank path end to end (replicas, universe sharding, weak field).
set -u
mkdir -p gpurun_out
PT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/dist2.log 2>&1 || exit $?
