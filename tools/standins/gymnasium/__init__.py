"""Minimal stand-in for `gymnasium` (absent in this image), used ONLY by tools/gen_golden.py to import
the reference for fixture generation. Provides just the names the reference touches."""
from . import spaces, wrappers  # noqa: F401


class Env:
    def close(self):
        pass


class Wrapper(Env):
    def __init__(self, env):
        self.env = env

    def __getattr__(self, item):
        return getattr(self.env, item)


class ObservationWrapper(Wrapper):
    pass
