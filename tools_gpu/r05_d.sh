#!/bin/bash
# Round 5 (d): the per-step exchange latency of a universe split over a team of workgroups (handoff_bench: leader +
# W-1 helpers on one XCD, sc1 hand-offs both ways per step, nothing else), and C3 with per-universe phase cycles.
set -u
mkdir -p gpurun_out
T=${TAG:-r05d}
timeout -k 10 60 ./tools_gpu/handoff_bench 3500 > gpurun_out/${T}_handoff.json 2> gpurun_out/${T}_handoff.err || exit $?
