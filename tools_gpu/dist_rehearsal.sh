#!/bin/bash
# N > 1 rehearsal of bench.py on a one-GPU box: `bench.py --gpus 2` started without a torch.distributed environment
# spawns its 2 ranks itself (torch.distributed.run, 127.0.0.1), here over gloo sharing the GPU (the driver runs N
# ranks over RCCL, one per GPU). Checks the multi-rank path end to end (replicas, universe sharding, weak and
# reference-scale fields) and that the line reports n_gpus 2.
set -u
mkdir -p gpurun_out
PT_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/dist2.log 2>&1 || exit $?
