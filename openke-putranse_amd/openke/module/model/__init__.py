from __future__ import absolute_import, division, print_function

from .Model import Model
from .TransE import TransE
from .TransH import TransH

__all__ = ['Model', 'TransE', 'TransH']
