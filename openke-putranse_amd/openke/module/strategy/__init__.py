from __future__ import absolute_import, division, print_function

from .Strategy import Strategy
from .NegativeSampling import NegativeSampling

__all__ = ['Strategy', 'NegativeSampling']
