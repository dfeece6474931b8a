"""Compat package `marl_factory_grid.utils.logging` (reference utils/logging/)."""
