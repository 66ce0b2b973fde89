#!/bin/bash
# Round 4 (z): the default bench line on the final build, now that profiles/pmc_c2.json is this library's profile
# (roofline.traffic / counted_frac must be filled, counters_match_build true)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r04z_default.log 2>&1 || exit $?
