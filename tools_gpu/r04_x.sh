#!/bin/bash
# Round 4 (x): the step-cost model with a per-positive part growing with the padded row (product) against the fixed
# 64 + bs model (ab/lib_p64.so) and the rounds model (ab/lib_old.so): C3 / C4 / C5, then the universe parity tests on
# the product.
set -u
TAG=r04x LIBS="old p64 prod" WLS="c3 c4 c5" STEPS=3 TESTLIB=prod bash tools_gpu/ab_libs.sh
