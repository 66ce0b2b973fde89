#!/bin/bash
# Round 4 (s): the hot kernels' phase B on half-width lane groups (ab/lib_bs.so) against the product: per-universe
# cycles on C3 / C4, then the universe parity tests on ab/lib_bs.so.
set -u
TAG=r04s LIBS="prod bs" WLS="c3 c4" STEPS=3 TESTLIB=bs bash tools_gpu/ab_libs.sh
