"""Compat module `marl_factory_grid.utils.tools` (reference utils/tools.py:21 ConfigExplainer)."""
import marl_factory_grid  # noqa: F401  (puts mfg_amd on sys.path)
from mfg_amd.explain import ConfigExplainer  # noqa: E402,F401
