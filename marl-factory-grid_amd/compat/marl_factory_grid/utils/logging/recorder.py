"""Compat module `marl_factory_grid.utils.logging.recorder` (reference utils/logging/recorder.py:10)."""
import marl_factory_grid  # noqa: F401  (puts mfg_amd on sys.path)
from mfg_amd.monitor import EnvRecorder  # noqa: E402,F401
