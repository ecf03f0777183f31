"""Gymnasium-compatible ``Box`` / ``Dict`` spaces for the façade (gymnasium is absent in this image).

When gymnasium is importable its own classes are used; otherwise these mirror the subset of
``gymnasium.spaces`` the reference's PickPlaceGymEnv exposes (gym_env.py:154-208): ``shape``,
``dtype``, ``low`` / ``high`` broadcast to the shape and cast to the dtype, ``sample()`` (uniform on
bounded dimensions, normal on unbounded ones, exponential on half-bounded ones, as gymnasium does),
``contains()``, ``seed()`` and, for ``Dict``, the ``spaces`` mapping in insertion order.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - gymnasium is not installed in this image
    from gymnasium.spaces import Box, Dict  # noqa: F401
except Exception:

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low) if np.ndim(low) else np.shape(high)
            self.shape = tuple(int(s) for s in shape)
            self.low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)
            if self.low.shape != self.shape or self.high.shape != self.shape:
                raise ValueError(f"low/high shape {self.low.shape}/{self.high.shape} != {self.shape}")
            self.np_random = np.random.default_rng(seed)

        def seed(self, seed=None):
            self.np_random = np.random.default_rng(seed)
            return [seed]

        def sample(self):
            lo, hi = self.low.astype(np.float64), self.high.astype(np.float64)
            out = np.empty(self.shape)
            bl, bh = np.isfinite(lo), np.isfinite(hi)
            both, none = bl & bh, ~bl & ~bh
            out[none] = self.np_random.normal(size=none.sum())
            out[bl & ~bh] = lo[bl & ~bh] + self.np_random.exponential(size=(bl & ~bh).sum())
            out[~bl & bh] = hi[~bl & bh] - self.np_random.exponential(size=(~bl & bh).sum())
            out[both] = self.np_random.uniform(lo[both], hi[both])
            if self.dtype.kind in "iu":
                out = np.floor(out)
            return out.astype(self.dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __contains__(self, x) -> bool:
            return self.contains(x)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Dict:
        def __init__(self, spaces: dict, seed=None):
            self.spaces = dict(spaces)
            for k, sp in enumerate(self.spaces.values()):
                sp.seed(None if seed is None else seed + k)

        def __getitem__(self, key):
            return self.spaces[key]

        def keys(self):
            return self.spaces.keys()

        def seed(self, seed=None):
            for k, sp in enumerate(self.spaces.values()):
                sp.seed(None if seed is None else seed + k)
            return [seed]

        def sample(self):
            return {k: sp.sample() for k, sp in self.spaces.items()}

        def contains(self, x) -> bool:
            return isinstance(x, dict) and set(x) == set(self.spaces) and all(
                self.spaces[k].contains(v) for k, v in x.items())

        def __contains__(self, x) -> bool:
            return self.contains(x)
