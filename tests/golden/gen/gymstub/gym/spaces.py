import numpy as np


class Discrete:
    def __init__(self, n):
        self.n = n

    def sample(self):
        return int(np.random.randint(self.n))


class Box:
    def __init__(self, low, high, shape=None, dtype=None):
        self.low, self.high, self.dtype = low, high, dtype
        self.shape = tuple(shape)
