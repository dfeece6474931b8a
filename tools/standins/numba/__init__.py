"""Stand-in: `njit` is the identity (the reference's @njit Bresenham is plain integer Python)."""


def njit(f=None, **kw):
    return f if f is not None else (lambda g: g)
