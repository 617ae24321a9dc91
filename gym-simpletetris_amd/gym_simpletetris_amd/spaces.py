"""Action/observation spaces.  Uses gym.spaces / gymnasium.spaces when one of
them is importable (the reference depends on gym>=0.21, setup.py:18); otherwise
minimal stand-ins with the same attributes (n / low / high / shape / dtype)."""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - neither is installed in the build image
    from gym import spaces as _sp  # type: ignore
except Exception:  # noqa: BLE001
    try:
        from gymnasium import spaces as _sp  # type: ignore
    except Exception:  # noqa: BLE001
        _sp = None


class _Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return int(rng.integers(0, self.n))

    def contains(self, x) -> bool:
        try:
            return 0 <= int(x) < self.n and int(x) == x
        except (TypeError, ValueError):
            return False

    def __repr__(self):
        return f"Discrete({self.n})"


class _Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def Discrete(n):
    return _sp.Discrete(n) if _sp is not None else _Discrete(n)


def Box(low, high, shape, dtype=np.float32):
    return _sp.Box(low, high, shape=shape, dtype=dtype) if _sp is not None else _Box(low, high, shape, dtype)
