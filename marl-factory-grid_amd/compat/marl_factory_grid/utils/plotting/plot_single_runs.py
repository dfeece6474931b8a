"""Compat module `marl_factory_grid.utils.plotting.plot_single_runs` (reference plot_single_runs.py:12)."""
import marl_factory_grid  # noqa: F401  (puts mfg_amd on sys.path)
from mfg_amd.plotting import plot_single_run  # noqa: E402,F401
