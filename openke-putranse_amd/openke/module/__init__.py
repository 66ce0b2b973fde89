from __future__ import absolute_import, division, print_function

from .BaseModule import BaseModule

__all__ = ['BaseModule']
