from __future__ import absolute_import, division, print_function

from .TrainDataLoader import TrainDataLoader
from .TestDataLoader import TestDataLoader

__all__ = ['TrainDataLoader', 'TestDataLoader']
