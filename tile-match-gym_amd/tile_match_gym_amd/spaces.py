"""Observation / action spaces.

Uses gymnasium.spaces when gymnasium is importable (the reference requires
gymnasium>=1.0.0, pyproject.toml:17).  This image has no gymnasium, so a
minimal stand-in with the same constructor signatures and the attributes the
reference reads (n, shape, dtype, low, high, spaces, seed, sample, contains)
is used instead.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium is installed
    from gymnasium.spaces import Box, Dict, Discrete, MultiDiscrete  # noqa: F401
    HAVE_GYMNASIUM = True
except Exception:  # gymnasium absent
    HAVE_GYMNASIUM = False

    class _Space:
        def __init__(self, shape=None, dtype=None, seed=None):
            self.shape = shape
            self.dtype = np.dtype(dtype) if dtype is not None else None
            self._np_random = None
            if seed is not None:
                self.seed(seed)

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.default_rng()
            return self._np_random

        def seed(self, seed=None):
            self._np_random = np.random.default_rng(seed)
            return [seed]

    class Discrete(_Space):
        def __init__(self, n, seed=None, start=0):
            self.n = int(n)
            self.start = int(start)
            super().__init__((), np.int64, seed)

        def sample(self, mask=None):
            return int(self.start + self.np_random.integers(self.n))

        def contains(self, x):
            try:
                x = int(x)
            except Exception:
                return False
            return self.start <= x < self.start + self.n

        def __repr__(self):
            return f"Discrete({self.n})"

        def __eq__(self, other):
            return isinstance(other, Discrete) and other.n == self.n and other.start == self.start

    class MultiDiscrete(_Space):
        """gymnasium.spaces.MultiDiscrete: one Discrete(nvec[i]) per entry, the
        batched form of Discrete (gymnasium.vector.utils.batch_space)."""

        def __init__(self, nvec, dtype=np.int64, seed=None, start=None):
            self.nvec = np.asarray(nvec, dtype=dtype)
            self.start = np.zeros_like(self.nvec) if start is None else np.asarray(start, dtype=dtype)
            super().__init__(self.nvec.shape, dtype, seed)

        def sample(self, mask=None):
            return (self.start + self.np_random.integers(0, self.nvec)).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.start)) and bool(np.all(x < self.start + self.nvec))

        def __repr__(self):
            return f"MultiDiscrete({self.nvec})"

        def __eq__(self, other):
            return isinstance(other, MultiDiscrete) and np.array_equal(other.nvec, self.nvec) and \
                np.array_equal(other.start, self.start)

    class Box(_Space):
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low) if np.ndim(low) else np.shape(high)
            shape = tuple(int(s) for s in shape)
            self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
            super().__init__(shape, dtype, seed)

        def sample(self, mask=None):
            if np.issubdtype(self.dtype, np.integer):
                return self.np_random.integers(self.low, self.high.astype(np.int64) + 1).astype(self.dtype)
            return self.np_random.uniform(self.low, self.high).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Dict(_Space):
        def __init__(self, spaces=None, seed=None, **kw):
            if spaces is None:
                spaces = {}
            spaces = dict(spaces, **kw)
            self.spaces = OrderedDict(spaces)
            super().__init__(None, None, None)
            if seed is not None:
                self.seed(seed)

        def __getitem__(self, key):
            return self.spaces[key]

        def keys(self):
            return self.spaces.keys()

        def seed(self, seed=None):
            for s in self.spaces.values():
                s.seed(seed)
            return [seed]

        def sample(self, mask=None):
            return OrderedDict((k, s.sample()) for k, s in self.spaces.items())

        def contains(self, x):
            return all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

        def __repr__(self):
            return "Dict(" + ", ".join(f"{k}: {v}" for k, v in self.spaces.items()) + ")"
