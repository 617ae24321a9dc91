"""ctypes wrapper around the C parity oracle (oracle/tetris_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  The oracle is a
cell-by-cell restatement of /root/reference/gym_simpletetris/envs/tetris_env.py
(TetrisEngine :125-335) + CPython's random; it is pinned by tests/golden/*.npz,
which were produced by running the reference itself (tests/golden/gen_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libtetris_oracle.so")

OR_MAX_W = 32
OR_MAX_H = 32
MT_N = 624

# Flag names in TetrisEngine.__init__ order (tetris_env.py:126-137).
SCORING_KEYS = ("reward_step", "penalise_height", "penalise_height_increase",
                "advanced_clears", "high_scoring", "penalise_holes",
                "penalise_holes_increase")


class MT(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * MT_N), ("index", ctypes.c_int32)]


class Config(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int32) for k in (
        "width", "height", "lock_delay", "step_reset") + SCORING_KEYS]


class Env(ctypes.Structure):
    _fields_ = [
        ("cfg", Config),
        ("board", (ctypes.c_uint8 * OR_MAX_H) * OR_MAX_W),
        ("shape", (ctypes.c_int32 * 2) * 4),
        ("shape_id", ctypes.c_int32),
        ("rot", ctypes.c_int32),
        ("ax", ctypes.c_int32),
        ("ay", ctypes.c_int32),
        ("lock", ctypes.c_int32),
        ("time", ctypes.c_int32),
        ("score", ctypes.c_int32),
        ("holes", ctypes.c_int32),
        ("lines_cleared", ctypes.c_int32),
        ("piece_height", ctypes.c_int32),
        ("n_deaths", ctypes.c_int32),
        ("counts", ctypes.c_int32 * 7),
        ("rng", MT),
    ]


def build(quiet: bool = True) -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    cmd = ["make", "-s", "-C", _HERE]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL if quiet else None)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.or_mt_seed_u64.argtypes = [ctypes.POINTER(MT), ctypes.c_uint64]
        L.or_mt_genrand.argtypes = [ctypes.POINTER(MT)]
        L.or_mt_genrand.restype = ctypes.c_uint32
        L.or_mt_randbelow.argtypes = [ctypes.POINTER(MT), ctypes.c_uint32]
        L.or_mt_randbelow.restype = ctypes.c_uint32
        L.or_env_init.argtypes = [ctypes.POINTER(Env), ctypes.POINTER(Config)]
        L.or_env_clear.argtypes = [ctypes.POINTER(Env)]
        L.or_env_step.argtypes = [ctypes.POINTER(Env), ctypes.c_int32, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        L.or_env_step.restype = ctypes.c_int32
        L.or_sizeof_env.restype = ctypes.c_int32
        L.or_batch_rollout.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.or_batch_rollout.restype = ctypes.c_int64
        assert L.or_sizeof_env() == ctypes.sizeof(Env), "oracle Env struct mismatch"
        _lib = L
    return _lib


def make_config(width=10, height=20, lock_delay=0, step_reset=False, **scoring) -> Config:
    unknown = set(scoring) - set(SCORING_KEYS)
    if unknown:
        raise TypeError(f"unknown kwargs {sorted(unknown)}")
    c = Config()
    c.width, c.height, c.lock_delay, c.step_reset = width, height, lock_delay, int(bool(step_reset))
    for k in SCORING_KEYS:
        setattr(c, k, int(bool(scoring.get(k, False))))
    return c


class MTRandom:
    """CPython random.Random restated (seed / getrandbits(32) / randint)."""

    def __init__(self, seed: int):
        self._mt = MT()
        lib().or_mt_seed_u64(ctypes.byref(self._mt), seed)

    def getrandbits32(self) -> int:
        return lib().or_mt_genrand(ctypes.byref(self._mt))

    def randint(self, a: int, b: int) -> int:
        return a + lib().or_mt_randbelow(ctypes.byref(self._mt), b - a + 1)


class OracleBatch:
    """N independent oracle envs (each with its own MT, reference R13/R14)."""

    def __init__(self, n: int, seeds, **kwargs):
        self.n = n
        self.cfg = make_config(**kwargs)
        self.envs = (Env * n)()
        L = lib()
        for i in range(n):
            L.or_env_init(ctypes.byref(self.envs[i]), ctypes.byref(self.cfg))
            L.or_mt_seed_u64(ctypes.byref(self.envs[i].rng), int(seeds[i]))

    def reset(self, i=None):
        L = lib()
        for k in (range(self.n) if i is None else [i]):
            L.or_env_clear(ctypes.byref(self.envs[k]))

    def step_one(self, i: int, action: int):
        """One reference step on env i -> (obs (W,H) u8, reward, done, rtype)."""
        W, H = self.cfg.width, self.cfg.height
        obs = np.zeros(W * H, np.uint8)
        done = ctypes.c_int32()
        rt = ctypes.c_int32()
        r = lib().or_env_step(ctypes.byref(self.envs[i]), int(action), obs.ctypes.data,
                              ctypes.byref(done), ctypes.byref(rt))
        return obs.reshape(W, H), r, bool(done.value), rt.value

    def rollout(self, actions: np.ndarray, want_obs=True, want_stats=True):
        """actions [T, n] u8 -> dict of per-step outputs; auto-resets on done."""
        actions = np.ascontiguousarray(actions, dtype=np.uint8)
        T = actions.shape[0]
        assert actions.shape[1] == self.n
        W = self.cfg.width
        rew = np.zeros((T, self.n), np.int32)
        done = np.zeros((T, self.n), np.uint8)
        obs = np.zeros((T, self.n, W), np.uint32) if want_obs else None
        st = np.zeros((T, self.n, 8), np.int32) if want_stats else None
        locks = lib().or_batch_rollout(
            ctypes.addressof(self.envs), self.n, T, actions.ctypes.data, rew.ctypes.data,
            done.ctypes.data, obs.ctypes.data if want_obs else None,
            st.ctypes.data if want_stats else None)
        return dict(reward=rew, done=done, obs=obs, stats=st, locks=int(locks))

    # ---- state access (crafted known-answer cases) ----
    def board(self, i) -> np.ndarray:
        W, H = self.cfg.width, self.cfg.height
        return np.ctypeslib.as_array(self.envs[i].board)[:W, :H].copy()

    def set_state(self, i, board=None, shape_id=None, rot=None, ax=None, ay=None, lock=None,
                  counts=None, **counters):
        e = self.envs[i]
        if board is not None:
            b = np.ctypeslib.as_array(e.board)
            b[:] = 0
            b[:board.shape[0], :board.shape[1]] = board
        if shape_id is not None:
            e.shape_id = shape_id
            cells = rotate_cells(BASE_SHAPES[shape_id], rot or 0)
            for c in range(4):
                e.shape[c][0], e.shape[c][1] = cells[c]
            e.rot = rot or 0
        if ax is not None:
            e.ax = ax
        if ay is not None:
            e.ay = ay
        if lock is not None:
            e.lock = lock
        if counts is not None:
            for k in range(7):
                e.counts[k] = int(counts[k])
        for k, v in counters.items():
            setattr(e, k, int(v))


# tetris_env.py:10-19, in shape_names order T,J,L,Z,S,I,O
BASE_SHAPES = (
    ((0, 0), (-1, 0), (1, 0), (0, -1)),
    ((0, 0), (-1, 0), (0, -1), (0, -2)),
    ((0, 0), (1, 0), (0, -1), (0, -2)),
    ((0, 0), (-1, 0), (0, -1), (1, -1)),
    ((0, 0), (-1, -1), (0, -1), (1, 0)),
    ((0, 0), (0, -1), (0, -2), (0, -3)),
    ((0, 0), (0, -1), (-1, 0), (-1, -1)),
)
SHAPE_NAMES = ("T", "J", "L", "Z", "S", "I", "O")


def rotate_cells(cells, rot):
    """rot applications of rotated(cclk=False) (tetris_env.py:22-26)."""
    cells = list(cells)
    for _ in range(rot % 4):
        cells = [(j, -i) for i, j in cells]
    return cells


def splitmix64_actions(seed: int, t0: int, steps: int, n: int, offset: int = 0) -> np.ndarray:
    """Synthetic action stream a[t,e] = splitmix64(seed ^ ((t << 32) ^ e)) % 7
    (SURVEY §8(d)); e is the GLOBAL env index (offset + local)."""
    with np.errstate(over="ignore"):
        t = (np.arange(t0, t0 + steps, dtype=np.uint64) << np.uint64(32))[:, None]
        e = np.arange(offset, offset + n, dtype=np.uint64)[None, :]
        z = np.uint64(seed) ^ (t ^ e)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(7)).astype(np.uint8)
