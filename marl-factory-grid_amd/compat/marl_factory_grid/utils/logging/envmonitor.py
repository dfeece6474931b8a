"""Compat module `marl_factory_grid.utils.logging.envmonitor` (reference utils/logging/envmonitor.py:14)."""
import marl_factory_grid  # noqa: F401  (puts mfg_amd on sys.path)
from mfg_amd.monitor import EnvMonitor  # noqa: E402,F401
