from __future__ import absolute_import, division, print_function

from .Trainer import Trainer
from .Tester import Tester
from .Validator import Validator
from .Parallel_Universe_Config import Parallel_Universe_Config

__all__ = ['Trainer', 'Tester', 'Parallel_Universe_Config', 'Validator']
