"""Compat package `marl_factory_grid.utils` (reference marl_factory_grid/utils/)."""
