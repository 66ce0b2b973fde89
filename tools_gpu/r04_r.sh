#!/bin/bash
# Round 4 (r): the hot single-shape kernels with the first negative's row prefetched (ab/lib_pf.so), with two
# phase-B rows per lane group for their shapes of at most 6 floats per lane (ab/lib_rb2.so), and both
# (ab/lib_pfrb.so), against the product: per-universe cycles on C3 / C4.
set -u
TAG=r04r LIBS="prod pf rb2 pfrb" WLS="c3 c4" STEPS=3 bash tools_gpu/ab_libs.sh
