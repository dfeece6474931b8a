"""Compat package `marl_factory_grid.utils.plotting` (reference utils/plotting/)."""
