#!/bin/bash
# Round 6 (s), closing evidence A on the final build: evidence A (r06_n.sh: GPU suite, chain counters, the driver's
# command and its kernel stats), then C2's PMC passes (pmc.sh).
set -u
TAG=${TAG:-r06s} bash tools_gpu/r06_n.sh || exit $?
bash tools_gpu/pmc.sh || exit $?
