#!/bin/bash
# Round 4 (w): the universe queue order (longest first by the step-cost model) with a fixed part of 24 positives
# (ab/lib_w24.so, C4's fit) against the product's 64 (C3's fit) and the pre-fit build (ab/lib_old.so): C4 / C3.
set -u
TAG=r04w LIBS="old prod w24" WLS="c4 c3" STEPS=3 bash tools_gpu/ab_libs.sh
