"""CPU oracle package — TEST INFRASTRUCTURE ONLY (see oracle.h). Never imported by the product."""
from .oracle import *  # noqa: F401,F403
