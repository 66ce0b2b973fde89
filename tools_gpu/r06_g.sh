#!/bin/bash
# Round 6 (g): instruction counts of the longest universe's chain (pmc_chain.sh) for C4 and C3, one workgroup and
# (C4) a team of 4.
set -u
W=c4 TW=1 bash tools_gpu/pmc_chain.sh && W=c3 TW=1 bash tools_gpu/pmc_chain.sh && W=c4 TW=4 bash tools_gpu/pmc_chain.sh
