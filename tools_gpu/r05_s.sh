#!/bin/bash
# Round 5 (s): synchronized phase times of the 512-universe drop-in, with and without the best-model checkpoints
set -u
mkdir -p gpurun_out
T=${TAG:-r05s}
timeout -k 10 300 python tools_gpu/dropin_phases.py c3 > gpurun_out/${T}_phases.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/dropin_phases.py c3 0 nosave > gpurun_out/${T}_phases_nosave.log 2>&1 || exit $?
