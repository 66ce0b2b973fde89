#!/bin/bash
# Round 4 (y): hot single-shape kernels for TransH too (product) against the final build (ab/lib_cur.so): C5 / C3, then
# the universe parity tests on the product.
set -u
TAG=r04y LIBS="cur prod" WLS="c5 c3" STEPS=3 TESTLIB=prod bash tools_gpu/ab_libs.sh
