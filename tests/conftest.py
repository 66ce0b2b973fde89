import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "openke-putranse_amd")
for p in (REPO, PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")
KG_SMALL = os.path.join(GOLDEN, "kg_small") + os.sep
KG_TINY = os.path.join(GOLDEN, "kg_tiny") + os.sep


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def pytest_collection_modifyitems(config, items):
    # a GPU-marked test must never silently pass on a box without a GPU: it is simply not collected
    # into the CPU run (-m "not gpu"); on the GPU box a missing device is a hard failure.
    pass
