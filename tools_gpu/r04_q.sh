#!/bin/bash
# Round 4 (q): paired presampling (product: a lane's two draws' loads in flight together) against the previous
# one-draw-at-a-time build (ab/lib_base.so) and against paired presampling plus the first negative's row
# prefetched in the hot single-shape kernels (ab/lib_pf.so): per-universe cycles on C3 / C4 / C5, then the
# universe parity tests on the product.
set -u
TAG=r04q LIBS="base prod pf" WLS="c3 c4 c5" STEPS=3 TESTLIB=prod bash tools_gpu/ab_libs.sh
