"""MI355X-native drop-in for the `openke` package of luofeisg/OpenKE-PuTransE (PuTransE / TransE /
TransH training and link prediction). Same import paths, class names, signatures and defaults as the
reference; the hot path runs in hand-written HIP kernels (release/libputranse_hip.so)."""
from __future__ import absolute_import, division, print_function
