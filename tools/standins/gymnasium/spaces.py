class Discrete:
    def __init__(self, n):
        self.n = int(n)


class Tuple(tuple):
    def __new__(cls, spaces):
        return super().__new__(cls, tuple(spaces))


class Box:
    def __init__(self, low, high, shape, dtype=None):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype
