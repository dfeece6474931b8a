"""Compat module for `marl_factory_grid.environment.factory` (reference environment/factory.py:21)."""
import os
import sys

_PKG = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..', '..'))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from mfg_amd.factory import Factory, BatchedFactory  # noqa: E402,F401
