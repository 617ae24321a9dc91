"""Golden-fixture replay harness shared by the oracle tests (CPU) and the HIP
parity tests (GPU).

An *adapter* wraps one batched engine and exposes:
    reset(mask)             -- TetrisEngine.clear() on envs where mask is True
    set_state(i, init)      -- load a crafted initial state (board/piece/counters)
    step(actions) -> dict   -- one reference step on every env, NO auto-reset;
                               returns per-env arrays keyed like Recorder.FIELDS
The replay loop mirrors the fixture driver in gen_golden.py: step all envs,
compare, then reset the envs that reported done (reference `if done: reset()`).
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
COMPARE = ("reward", "done", "time", "score", "lines", "holes", "deaths", "piece", "height",
           "counts", "obs", "board")


def load_set(fname):
    d = np.load(os.path.join(GOLDEN, fname))
    meta = json.loads(str(d["meta"]))
    out = {}
    for name, m in meta.items():
        arrs = {k.split("/", 1)[1]: d[k] for k in d.files if k.startswith(name + "/")}
        out[name] = (m, arrs)
    return out


def engine_kwargs(cfg):
    kw = dict(width=10, height=20, lock_delay=0, step_reset=False)
    kw.update(cfg)
    return kw


def _check(name, t, got, exp, fields, env_slice=slice(None)):
    for k in fields:
        if k not in got:
            continue
        g = np.asarray(got[k])
        x = np.asarray(exp[k])[t][env_slice] if np.asarray(exp[k]).ndim > 1 else np.asarray(exp[k])[t]
        if g.shape != x.shape or not np.array_equal(g, x.astype(g.dtype)):
            bad = np.argwhere(np.asarray(g != x.astype(g.dtype)).reshape(g.shape[0], -1).any(1)).ravel() \
                if g.ndim >= 1 and g.shape == x.shape else None
            raise AssertionError(f"{name}: step {t} field {k!r} mismatch (envs {bad}):\n"
                                 f"got {g if g.size < 64 else g[bad] if bad is not None else g}\n"
                                 f"exp {x if x.size < 64 else x[bad] if bad is not None else x}")


def replay_rollout(adapter_factory, name, meta, arrs, fields=COMPARE, steps=None):
    n = meta["n_envs"]
    seeds = [meta["seed_base"] + e for e in range(n)]
    ad = adapter_factory(n, seeds, engine_kwargs(meta["cfg"]))
    ad.reset(np.ones(n, bool))
    T = arrs["actions"].shape[0] if steps is None else min(steps, arrs["actions"].shape[0])
    for t in range(T):
        got = ad.step(arrs["actions"][t])
        _check(name, t, got, arrs, fields)
        done = np.asarray(got["done"]).astype(bool)
        if done.any():
            ad.reset(done)
    return T * n


def replay_crafted(adapter_factory, name, meta, arrs, fields=COMPARE):
    ad = adapter_factory(1, [meta["seed"]], engine_kwargs(meta["cfg"]))
    ad.reset(np.ones(1, bool))
    init = {k[5:]: arrs[k] for k in arrs if k.startswith("init_")}
    ad.set_state(0, init)
    for t, a in enumerate(meta["actions"]):
        got = ad.step(np.array([a], np.uint8))
        exp = {k: arrs[k][t:t + 1] for k in fields if k in arrs}
        _check(name, 0, {k: v for k, v in got.items()}, {k: v[None] for k, v in exp.items()}, fields)
        if got["done"][0] and not meta["no_reset"]:
            ad.reset(np.ones(1, bool))


def unpack_piece(p):
    p = np.asarray(p, np.uint32)
    return dict(id=p & 7, rot=(p >> 3) & 3, ax=(p >> 5) & 63, ay=(p >> 11) & 63, lock=p >> 17)
