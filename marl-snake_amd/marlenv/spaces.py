"""Minimal gym-style spaces (gym itself is not a dependency of this package).

Mirrors what the reference reads from gym.spaces (snake_env.py:107-129,
wrappers.py:88-97,111-124): ``.n``/``.sample()`` of Discrete and
``.shape``/``.dtype``/``.low``/``.high`` of Box. Each space samples from its own
numpy Generator, like gym's per-space np_random, so sampling never perturbs the
global legacy RandomState the env's compat mode follows.
"""
import numpy as np


class Discrete:
    def __init__(self, n, seed=None):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64
        self._rng = np.random.default_rng(seed)

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        return int(self._rng.integers(self.n))

    def contains(self, x):
        try:
            return 0 <= int(x) < self.n and float(x) == int(x)
        except (TypeError, ValueError):
            return False

    def __repr__(self):
        return f'Discrete({self.n})'

    def __eq__(self, other):
        return isinstance(other, Discrete) and other.n == self.n


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.low, self.high = low, high
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return self._rng.integers(self.low, self.high, size=self.shape, endpoint=True).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

    def __repr__(self):
        return f'Box({self.low}, {self.high}, {self.shape}, {self.dtype})'
