"""Generate the golden parity fixtures by running the REFERENCE itself.

Runs only in the build container (needs /root/reference, read-only).  The
reference module gym_simpletetris/envs/tetris_env.py is loaded unmodified by
file path with three workarounds: stub `gym`/`gym.spaces`/
`pygame` modules (not installed; they only feed the spaces metadata and the
human renderer) and `np.float = float` (tetris_env.py:140 uses the alias
removed in numpy >= 1.24).  Nothing from the reference is copied: only its
outputs (inputs + expected outputs) are written as .npz data.

Multi-env isolation protocol: the reference draws pieces from
the GLOBAL CPython `random` (tetris_env.py:187); env e "with seed s_e" is
defined as `random.seed(s_e)` before its first reset, and every reset/step of
env e runs between `random.setstate(state_e)` and `state_e = random.getstate()`.

Fixtures:
  mt19937.npz          F4  CPython random known answers (words + randint draws)
  rollouts.npz         F1  uniform (splitmix64) action rollouts, several configs
  greedy.npz           F2  greedy-placement rollouts (1-4 line clears)
  crafted.npz          F3  crafted known-answer cases per reference rule
  grayscale.npz        F5  convert_grayscale images (next row, R19)
  render.npz           F5b engine.render(), render("rgb_array") and grayscale/rgb obs
                           along uniform-action games (python gen_golden.py render)

Usage: python tests/golden/gen_golden.py  (writes next to this file)
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/gym_simpletetris/envs/tetris_env.py"
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.oracle import splitmix64_actions, BASE_SHAPES, rotate_cells  # noqa: E402


def load_reference():
    sys.dont_write_bytecode = True
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Env:  # gym.Env stand-in; only subclassed
        pass

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Box:
        def __init__(self, low, high, shape=None, dtype=None):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    gym.Env, spaces.Discrete, spaces.Box, gym.spaces = Env, Discrete, Box, spaces
    sys.modules.setdefault("gym", gym)
    sys.modules.setdefault("gym.spaces", spaces)
    sys.modules.setdefault("pygame", types.ModuleType("pygame"))
    np.float = float  # tetris_env.py:140
    spec = importlib.util.spec_from_file_location("ref_tetris_env", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ref = None

SHAPE_NAMES = ["T", "J", "L", "Z", "S", "I", "O"]
KW_KEYS = ("width", "height", "lock_delay", "step_reset", "reward_step", "penalise_height",
           "penalise_height_increase", "advanced_clears", "high_scoring", "penalise_holes",
           "penalise_holes_increase")


def rtype_code(r):
    if type(r) is int:
        return 0
    if type(r) is np.int64:
        return 1
    if type(r) is float:
        return 2
    if type(r) is np.float64:
        return 3
    raise TypeError(type(r))


def ref_rot(engine):
    """Recover (id, rot) of the engine's current cell list."""
    sid = SHAPE_NAMES.index(engine.shape_name)
    cells = [tuple(c) for c in engine.shape]
    for r in range(4):
        if [tuple(c) for c in rotate_cells(BASE_SHAPES[sid], r)] == cells:
            return sid, r
    raise AssertionError("unrecognised rotation")


def pack_piece(engine):
    sid, rot = ref_rot(engine)
    ax, ay = int(engine.anchor[0]), int(engine.anchor[1])
    return sid | (rot << 3) | (ax << 5) | (ay << 11) | (int(engine._lock_delay) << 17)


def pack_cols(board):
    """board (W,H) 0/1 -> u32[W], bit y of word x."""
    b = (np.asarray(board) != 0).astype(np.uint64)
    w = (b << np.arange(b.shape[1], dtype=np.uint64)[None, :]).sum(axis=1)
    return w.astype(np.uint32)


class Recorder:
    FIELDS = ("reward", "rtype", "done", "time", "score", "lines", "holes", "deaths",
              "piece", "height", "counts", "obs", "board")

    def __init__(self):
        self.rows = {k: [] for k in self.FIELDS}

    def add(self, env, obs, reward, done, info):
        eng = env.engine
        self.rows["reward"].append(int(reward))
        assert float(reward) == int(reward)
        self.rows["rtype"].append(rtype_code(reward))
        self.rows["done"].append(int(done))
        self.rows["time"].append(int(info["time"]))
        self.rows["score"].append(int(info["score"]))
        self.rows["lines"].append(int(info["lines_cleared"]))
        self.rows["holes"].append(int(info["holes"]))
        self.rows["deaths"].append(int(info["deaths"]))
        self.rows["piece"].append(pack_piece(eng))
        self.rows["height"].append(int(eng.piece_height))
        self.rows["counts"].append([int(eng.shape_counts[k]) for k in SHAPE_NAMES])
        self.rows["obs"].append(pack_cols(obs))
        self.rows["board"].append(pack_cols(eng.board))


def make_env(cfg):
    kw = {k: v for k, v in cfg.items() if k in KW_KEYS}
    return ref.TetrisEnv(**kw)


# ---------------------------------------------------------------- F4
def gen_mt():
    seeds = [0, 1, 42, 12345, 2**31 - 1, 2**32 - 1, 2**32, 2**32 + 5, 2**63 + 123, 2**64 - 1]
    words, draws = [], []
    ns = np.arange(35, 98, dtype=np.int64)
    for s in seeds:
        r = random.Random(s)
        words.append([r.getrandbits(32) for _ in range(1500)])
        r = random.Random(s)
        draws.append([r.randint(1, int(ns[i % len(ns)])) for i in range(1500)])
    np.savez_compressed(os.path.join(HERE, "mt19937.npz"),
                        seeds=np.array(seeds, dtype=np.uint64),
                        words=np.array(words, dtype=np.uint32),
                        draws=np.array(draws, dtype=np.int32), ns=ns)


# ---------------------------------------------------------------- F1/F2
CONFIGS = {
    "default": {},
    "adv_holes_height": dict(advanced_clears=True, penalise_holes_increase=True,
                             penalise_height_increase=True),
    "high_height_holes": dict(high_scoring=True, penalise_height=True, penalise_holes=True),
    "reward_step": dict(reward_step=True),
    "lock2_reset": dict(lock_delay=2, step_reset=True),
    "lock3": dict(lock_delay=3, penalise_holes_increase=True),
    "small_odd": dict(width=7, height=12, penalise_holes=True, reward_step=True),
    "tall_wide": dict(width=13, height=26, penalise_height_increase=True, advanced_clears=True),
}


def greedy_target(eng):
    """Best (rot, x) for the current piece by hard-drop placement heuristic."""
    sid, _ = ref_rot(eng)
    W, H = eng.width, eng.height
    best, best_s = None, -1e18
    for rot in range(4):
        cells = rotate_cells(BASE_SHAPES[sid], rot)
        for x in range(-3, W + 3):
            if ref.is_occupied(cells, (x, 0), eng.board):
                continue
            y = 0
            while not ref.is_occupied(cells, (x, y + 1), eng.board):
                y += 1
            b = eng.board.copy()
            ok = True
            for i, j in cells:
                if 0 <= x + i < W and 0 <= y + j < H:
                    b[x + i, y + j] = 1
                elif y + j < 0:
                    ok = False
            full = int(np.all(b, axis=0).sum())
            keep = b[:, ~np.all(b, axis=0)]
            nb = np.zeros_like(b)
            nb[:, H - keep.shape[1]:] = keep
            holes = np.count_nonzero(nb.cumsum(axis=1) * ~nb.astype(bool))
            filled_rows = np.any(nb, axis=0)
            height = H - int(np.argmax(filled_rows)) if filled_rows.any() else 0
            s = 40 * full - 6 * holes - 1.5 * height - (1000 if not ok else 0)
            if s > best_s:
                best_s, best = s, (rot, x)
    return best


def greedy_action(eng, target, rng):
    if rng.random() < 0.03:
        return int(rng.integers(0, 7))
    if target is None:
        return 2
    sid, rot = ref_rot(eng)
    trot, tx = target
    if rot != trot:
        return 4
    ax = int(eng.anchor[0])
    if ax < tx:
        return 1
    if ax > tx:
        return 0
    return 2


def run_rollouts(n_envs, steps, cfg, seed_base, action_seed, policy):
    envs = [make_env(cfg) for _ in range(n_envs)]
    states = []
    for e in range(n_envs):
        random.seed(seed_base + e)
        envs[e].reset()
        states.append(random.getstate())
    rec = [Recorder() for _ in range(n_envs)]
    acts = np.zeros((steps, n_envs), np.uint8)
    if policy == "uniform":
        acts[:] = splitmix64_actions(action_seed, 0, steps, n_envs)
    prng = np.random.default_rng(action_seed)
    targets = [None] * n_envs
    last_total = [-1] * n_envs
    for t in range(steps):
        for e in range(n_envs):
            env = envs[e]
            random.setstate(states[e])
            if policy == "greedy":
                tot = sum(env.engine.shape_counts.values())
                if tot != last_total[e]:
                    targets[e] = greedy_target(env.engine)
                    last_total[e] = tot
                acts[t, e] = greedy_action(env.engine, targets[e], prng)
            obs, r, d, info = env.step(int(acts[t, e]))
            rec[e].add(env, obs, r, d, info)
            if d:
                env.reset()
            states[e] = random.getstate()
    out = {"actions": acts}
    for k in Recorder.FIELDS:
        out[k] = np.stack([np.array(rec[e].rows[k]) for e in range(n_envs)], axis=1)
    return out


def save_rollout_set(fname, policy, n_envs, steps, names):
    blob, meta = {}, {}
    for name in names:
        cfg = CONFIGS[name]
        seed_base = 1000 + 97 * len(meta)
        action_seed = 0xC0FFEE + len(meta)
        d = run_rollouts(n_envs, steps, cfg, seed_base, action_seed, policy)
        for k, v in d.items():
            dt = {"reward": np.int32, "rtype": np.uint8, "done": np.uint8, "piece": np.uint32,
                  "obs": np.uint32, "board": np.uint32, "actions": np.uint8}.get(k, np.int32)
            blob[f"{name}/{k}"] = v.astype(dt)
        meta[name] = dict(cfg=cfg, seed_base=seed_base, action_seed=action_seed,
                          n_envs=n_envs, steps=steps, policy=policy,
                          lines=int(d["lines"][-1].sum()), dones=int(d["done"].sum()))
        print(fname, name, meta[name]["lines"], "lines", meta[name]["dones"], "dones")
    blob["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, fname), **blob)


# ---------------------------------------------------------------- F3
def board_from_rows(W, H, rows):
    """rows: dict y -> string of W chars ('#' filled, '.' empty)."""
    b = np.zeros((W, H))
    for y, s in rows.items():
        assert len(s) == W
        for x, ch in enumerate(s):
            b[x, y] = 1.0 if ch == "#" else 0.0
    return b


def crafted_cases():
    W, H = 10, 20
    cases = []
    # 1. O hard-drop double clear under each scoring variant.
    dbl = board_from_rows(W, H, {18: "####..####", 19: "####..####", 17: "#.........",
                                 16: "#........."})
    for name, cfg in [("dbl_default", {}), ("dbl_reward_step", dict(reward_step=True)),
                      ("dbl_advanced", dict(advanced_clears=True)),
                      ("dbl_high", dict(high_scoring=True)),
                      ("dbl_pen_height", dict(penalise_height=True)),
                      ("dbl_pen_holes_inc", dict(penalise_holes_increase=True)),
                      ("dbl_pen_height_inc", dict(penalise_height_increase=True)),
                      ("dbl_adv_pen_height", dict(advanced_clears=True, penalise_height=True))]:
        cases.append(dict(name=name, cfg=cfg, seed=7, board=dbl, shape=6, rot=0, ax=5, ay=0,
                          counters=dict(holes=0, piece_height=4), actions=[2, 6, 6]))
    # 2. a clear removes a covered hole -> penalise_holes_increase gives a bonus.
    hole = board_from_rows(W, H, {15: "##########", 16: "#.########", 17: "#########.",
                                  18: "#########.", 19: "#########."})
    cases.append(dict(name="hole_removed", cfg=dict(penalise_holes_increase=True), seed=11,
                      board=hole, shape=5, rot=0, ax=9, ay=0,
                      counters=dict(holes=1), actions=[2, 6]))
    # 3. death-step erase (R8), continue stepping without reset.
    top = {y: "#########." for y in range(1, 20)}
    top[0] = "........#."
    death = board_from_rows(W, H, top)
    cases.append(dict(name="death_erase", cfg={}, seed=3, board=death, shape=6, rot=0, ax=5,
                      ay=0, counters={}, actions=[6, 0, 1, 6, 2], no_reset=True))
    # 4. S hanging off the left edge above the board.
    cases.append(dict(name="s_hang_left", cfg={}, seed=5, board=np.zeros((W, H)), shape=4,
                      rot=0, ax=1, ay=0, counters={}, actions=[0, 0, 6, 4, 0, 5, 0, 2]))
    # 5. O rotation drift.
    cases.append(dict(name="o_rotation_drift", cfg={}, seed=9, board=np.zeros((W, H)),
                      shape=6, rot=0, ax=5, ay=0, counters={},
                      actions=[4, 4, 4, 4, 5, 5, 1, 1, 1, 1, 4, 2]))
    # 6. lock_delay=2 trace at the floor.
    cases.append(dict(name="lock_delay2", cfg=dict(lock_delay=2), seed=13,
                      board=np.zeros((W, H)), shape=0, rot=0, ax=4, ay=16, counters={},
                      actions=[6, 6, 6, 6, 6, 6, 6, 6]))
    # 7. lock_delay=2 + step_reset: slide off a ledge resets the counter.
    ledge = board_from_rows(W, H, {18: "#####.....", 19: "#####....."})
    cases.append(dict(name="lock_delay_step_reset", cfg=dict(lock_delay=2, step_reset=True),
                      seed=17, board=ledge, shape=6, rot=0, ax=2, ay=16, counters={},
                      actions=[6, 1, 1, 1, 1, 6, 6, 6, 6, 6]))
    # 8. 4-line Tetris with a vertical I into a well.
    well = board_from_rows(W, H, {y: "###.######" for y in range(16, 20)})
    for name, cfg in [("tetris_default", {}), ("tetris_advanced", dict(advanced_clears=True)),
                      ("tetris_adv_all", dict(advanced_clears=True, penalise_height_increase=True,
                                              penalise_holes_increase=True, reward_step=True))]:
        cases.append(dict(name=name, cfg=cfg, seed=21, board=well, shape=5, rot=0, ax=3, ay=0,
                          counters=dict(piece_height=4), actions=[2, 6, 6]))
    # 9. rotation blocked by the wall / by blocks (no kicks).
    wall = board_from_rows(W, H, {y: "#........." for y in range(10, 20)})
    cases.append(dict(name="rot_blocked", cfg={}, seed=23, board=wall, shape=5, rot=1, ax=4,
                      ay=8, counters={}, actions=[0, 0, 0, 0, 5, 4, 4, 1, 4, 2]))
    # 10. hard drop onto an overhang / into a covered slot.
    ov = board_from_rows(W, H, {12: "...####...", 19: "##.#######", 18: "##.#######"})
    cases.append(dict(name="overhang", cfg=dict(penalise_holes=True), seed=29, board=ov,
                      shape=5, rot=0, ax=4, ay=3, counters={}, actions=[2, 0, 0, 0, 2, 6]))
    # 11. triple clear with non-contiguous full rows (compaction order).
    tri = board_from_rows(W, H, {16: "####.#####", 17: "#.#.######", 18: "####.#####",
                                 19: "####.#####"})
    cases.append(dict(name="split_clear", cfg=dict(penalise_height_increase=True), seed=31,
                      board=tri, shape=5, rot=0, ax=4, ay=0, counters=dict(piece_height=4),
                      actions=[2, 6, 6, 6]))
    # 12. right edge, I horizontal near the wall.
    cases.append(dict(name="right_edge", cfg={}, seed=37, board=np.zeros((W, H)), shape=5,
                      rot=3, ax=6, ay=5, counters={}, actions=[1, 1, 1, 0, 5, 1, 1, 1, 2]))
    return cases


def run_crafted(case):
    env = make_env(case["cfg"])
    random.seed(case["seed"])
    env.reset()
    eng = env.engine
    W, H = eng.width, eng.height
    eng.board = case["board"].astype(float).copy()
    eng.shape_name = SHAPE_NAMES[case["shape"]]
    eng.shape = [tuple(c) for c in rotate_cells(BASE_SHAPES[case["shape"]], case["rot"])]
    eng.anchor = (case["ax"], case["ay"])
    assert not ref.is_occupied(eng.shape, eng.anchor, eng.board), case["name"]
    for k, v in case["counters"].items():
        setattr(eng, k, v)
    init = dict(board=pack_cols(eng.board), piece=pack_piece(eng), time=eng.time,
                score=eng.score, lines=eng.lines_cleared, holes=eng.holes,
                height=eng.piece_height, deaths=eng.n_deaths,
                counts=[eng.shape_counts[k] for k in SHAPE_NAMES],
                mt_state=list(random.getstate()[1]))
    rec = Recorder()
    for a in case["actions"]:
        obs, r, d, info = env.step(a)
        rec.add(env, obs, r, d, info)
        if d and not case.get("no_reset"):
            env.reset()
    return init, rec


def gen_crafted():
    blob, meta = {}, {}
    for case in crafted_cases():
        init, rec = run_crafted(case)
        n = case["name"]
        meta[n] = dict(cfg=case["cfg"], seed=case["seed"], no_reset=bool(case.get("no_reset")),
                       actions=case["actions"])
        for k in ("board", "piece", "time", "score", "lines", "holes", "height", "deaths",
                  "counts"):
            blob[f"{n}/init_{k}"] = np.asarray(init[k]).astype(
                np.uint32 if k in ("board", "piece") else np.int32)
        blob[f"{n}/init_mt"] = np.asarray(init["mt_state"], dtype=np.uint64)
        for k in Recorder.FIELDS:
            dt = {"reward": np.int32, "rtype": np.uint8, "done": np.uint8, "piece": np.uint32,
                  "obs": np.uint32, "board": np.uint32}.get(k, np.int32)
            blob[f"{n}/{k}"] = np.array(rec.rows[k]).astype(dt)
        print("crafted", n, "rewards", rec.rows["reward"])
    blob["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, "crafted.npz"), **blob)


# ---------------------------------------------------------------- F5
def gen_grayscale():
    rng = np.random.default_rng(5)
    boards, g84, g160, dims = [], [], [], []
    for W, H in [(10, 20), (10, 20), (10, 20), (10, 20), (7, 12), (13, 26), (20, 10), (8, 8)]:
        b = (rng.random((W, H)) < 0.35).astype(float)
        pad = np.zeros((32, 32), np.uint8)
        pad[:W, :H] = b
        boards.append(pad)
        dims.append((W, H))
        g84.append(ref.convert_grayscale(b, 84))
        g160.append(ref.convert_grayscale(b, 160))
    np.savez_compressed(os.path.join(HERE, "grayscale.npz"), boards=np.array(boards),
                        dims=np.array(dims, np.int32), g84=np.array(g84, np.uint8),
                        g160=np.array(g160, np.uint8))


# ---------------------------------------------------------------- F5b
RENDER_RUNS = (("default", dict(), 4242), ("small_odd", dict(width=7, height=12), 4343),
               ("tall_wide", dict(width=13, height=26), 4444))
RENDER_AT = (0, 3, 11, 40, 77, 120, 199)


def gen_render():
    """engine.render() (tetris_env.py:317-321), env.render('rgb_array')
    (:458-462) and the 'grayscale' / 'rgb' observations (:413-433) along
    uniform-action games: one env per obs_type, same seed and actions, so the
    three runs see the same boards."""
    blob, meta = {}, {}
    steps = max(RENDER_AT) + 1
    for name, cfg, seed in RENDER_RUNS:
        acts = splitmix64_actions(0xBEEF, 0, steps, 1)[:, 0]
        envs = {}
        states = {}
        for ot in ("ram", "grayscale", "rgb"):
            envs[ot] = ref.TetrisEnv(obs_type=ot, **cfg)
            random.seed(seed)
            o = envs[ot].reset()
            states[ot] = random.getstate()
        packed, rgb, gray, rgbobs = [], [], [], []
        for t in range(steps):
            obs = {}
            for ot, env in envs.items():
                random.setstate(states[ot])
                o, r, d, info = env.step(int(acts[t]))
                obs[ot] = o
                if d:
                    env.reset()
                states[ot] = random.getstate()
            if t in RENDER_AT:
                e = envs["ram"]
                packed.append(pack_cols(e.engine.render()))
                img = e.render("rgb_array")
                assert img.dtype == np.uint8 and img.shape == (160, 160, 3)
                assert (img == img[:, :, :1]).all()
                rgb.append(img[:, :, 0])
                g = obs["grayscale"]
                assert g.dtype == np.float32 and g.shape == (84, 84)
                gray.append(g.astype(np.uint8))
                c = obs["rgb"]
                assert c.shape == (84, 84, 3) and (c == c[:, :, :1]).all()
                assert np.array_equal(c[:, :, 0], g)
                rgbobs.append(c[:, :, 0].astype(np.uint8))
        blob[f"{name}/actions"] = acts.astype(np.uint8)
        blob[f"{name}/render"] = np.array(packed, np.uint32)
        blob[f"{name}/rgb160"] = np.array(rgb, np.uint8)
        blob[f"{name}/gray84"] = np.array(gray, np.uint8)
        meta[name] = dict(cfg=cfg, seed=seed, at=list(RENDER_AT))
        print("render", name, len(packed), "frames")
    blob["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, "render.npz"), **blob)


GENERATORS = ("mt", "crafted", "rollouts", "greedy", "grayscale", "render")


def main(which=GENERATORS):
    global ref
    if not os.path.exists(REF):
        raise SystemExit("reference not present; fixtures are committed, nothing to do")
    ref = load_reference()
    if "render" in which:
        gen_render()
    if not set(which) - {"render"}:
        return
    gen_mt()
    gen_crafted()
    save_rollout_set("rollouts.npz", "uniform", 16, 400, list(CONFIGS))
    save_rollout_set("greedy.npz", "greedy", 8, 800,
                     ["default", "adv_holes_height", "high_height_holes", "reward_step",
                      "lock2_reset", "small_odd"])
    gen_grayscale()


if __name__ == "__main__":
    # no arguments: every fixture; else a subset of GENERATORS (only "render"
    # is generated on its own, the others are written together)
    main(tuple(sys.argv[1:]) or GENERATORS)
