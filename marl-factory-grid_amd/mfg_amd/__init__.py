"""mfg_amd — MI355X-native batched step engine for the marl-factory-grid world.

Host side (Python): spec compiler (spec.py), HIP engine binding (engine.py: Engine, PackedObs),
reference-compatible single-env facade and the batched env (factory.py: Factory, BatchedFactory), vector-env
adapters (vec.py), info rebuild (info.py, info_columns.py), entity views (views.py), on-GPU MARL training over
packed observations (marl.py).
Device side: csrc/mfg_engine.hip -> _lib/libmfg_hip.so (C-ABI: include/mfg.h).
"""
from .spec import compile_spec, EnvSpec, UnsupportedSpec  # noqa: F401

__all__ = ['compile_spec', 'EnvSpec', 'UnsupportedSpec']
