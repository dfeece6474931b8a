"""mfg_amd — MI355X-native batched step engine for the marl-factory-grid world.

Host side (Python): spec compiler (spec.py), HIP engine binding (engine.py), batched vector env
(batched.py), reference-compatible single-env facade (factory.py), info rebuild (info.py).
Device side: csrc/mfg_engine.hip -> _lib/libmfg_hip.so (C-ABI: include/mfg.h).
"""
from .spec import compile_spec, EnvSpec, UnsupportedSpec  # noqa: F401

__all__ = ['compile_spec', 'EnvSpec', 'UnsupportedSpec']
