"""Argument-recording stand-ins for gym.spaces (golden generation only)."""


class _Space(object):
    def __init__(self, *args, **kwargs):
        self.args = args
        self.kwargs = kwargs


class Box(_Space):
    def __init__(self, low=None, high=None, shape=None, dtype=None, **kwargs):
        super().__init__(low, high, shape, dtype, **kwargs)
        self.shape = shape
        self.dtype = dtype


class Discrete(_Space):
    def __init__(self, n):
        super().__init__(n)
        self.n = n


class Tuple(_Space):
    def __init__(self, spaces):
        super().__init__(spaces)
        self.spaces = spaces
