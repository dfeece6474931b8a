"""Compat import path: `from marl_factory_grid import Factory` resolves to the MI355X engine's facade
(mfg_amd.factory.Factory), so reference scripts run unchanged with `marl-factory-grid_amd/compat` on
sys.path. Only the stepping API is provided (quickstart/CLI are out of scope)."""
from marl_factory_grid.environment.factory import Factory  # noqa: F401
