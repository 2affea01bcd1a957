"""Minimal gym-0.21-compatible spaces (gym is not a dependency).

Only what the reference env surface uses: ``Box``, ``Dict`` (plain-dict input
is key-sorted, as gym 0.21 does), ``Tuple`` and ``MultiDiscrete`` with
``contains`` / ``sample`` / ``shape`` (reference masurvival_env.py:391-453,
demo.py:18-22).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional

import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None, seed: Optional[int] = None):
        self.shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]

    def __contains__(self, x):
        return self.contains(x)


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        super().__init__(shape, dtype, seed)
        self.low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)

    def contains(self, x) -> bool:
        if not isinstance(x, np.ndarray):
            x = np.asarray(x, dtype=self.dtype)
        return bool(np.can_cast(x.dtype, self.dtype) and x.shape == self.shape and np.all(x >= self.low)
                    and np.all(x <= self.high))

    def sample(self):
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return self.np_random.uniform(lo, hi).astype(self.dtype)

    def __repr__(self):
        return f'Box({self.shape}, {self.dtype})'


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64, seed=None):
        self.nvec = np.asarray(nvec, dtype=dtype)
        super().__init__(self.nvec.shape, dtype, seed)

    def contains(self, x) -> bool:
        if isinstance(x, list):
            x = np.array(x)
        x = np.asarray(x)
        return bool(x.shape == self.shape and x.dtype != object and np.all(0 <= x) and np.all(x < self.nvec))

    def sample(self):
        return (self.np_random.random(self.nvec.shape) * self.nvec).astype(self.dtype)

    def __repr__(self):
        return f'MultiDiscrete({self.nvec})'


class Tuple(Space):
    def __init__(self, spaces, seed=None):
        self.spaces = tuple(spaces)
        super().__init__(None, None, seed)

    def contains(self, x) -> bool:
        if isinstance(x, list):
            x = tuple(x)
        return isinstance(x, tuple) and len(x) == len(self.spaces) and all(
            s.contains(p) for s, p in zip(self.spaces, x))

    def sample(self):
        return tuple(s.sample() for s in self.spaces)

    def seed(self, seed=None):
        for k, s in enumerate(self.spaces):
            s.seed(None if seed is None else seed + k)
        return [seed]

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)

    def __iter__(self):
        return iter(self.spaces)


class Dict(Space):
    def __init__(self, spaces=None, seed=None):
        if isinstance(spaces, dict) and not isinstance(spaces, OrderedDict):
            spaces = OrderedDict(sorted(spaces.items()))
        self.spaces = OrderedDict(spaces)
        super().__init__(None, None, seed)

    def contains(self, x) -> bool:
        if not isinstance(x, dict) or len(x) != len(self.spaces):
            return False
        for k, s in self.spaces.items():
            if k not in x or not s.contains(x[k]):
                return False
        return True

    def sample(self):
        return OrderedDict((k, s.sample()) for k, s in self.spaces.items())

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def __iter__(self):
        return iter(self.spaces)

    def __repr__(self):
        return 'Dict(' + ', '.join(f'{k}: {s}' for k, s in self.spaces.items()) + ')'
