from __future__ import absolute_import, division, print_function

from .Loss import Loss
from .MarginLoss import MarginLoss

__all__ = ['Loss', 'MarginLoss']
