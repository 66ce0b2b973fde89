#!/bin/bash
# Round 5 (f): host profile of the drop-in C3 leg
set -u
mkdir -p gpurun_out
T=${TAG:-r05f}
timeout -k 10 300 python tools_gpu/prof_dropin.py c3 > gpurun_out/${T}_prof_c3.txt 2>&1 || exit $?
