"""Gym surface of SimpleTetris-v0 on the MI355X engine.

TetrisEnv     -- the reference's single-env class (tetris_env.py:338-467):
                 same constructor kwargs, spaces, step/reset/render/close,
                 numpy float32 observations, the reference's reward *types*
                 (int / np.int64 / float / np.float64, R18) and info dict.
                 By default its pieces come from CPython's GLOBAL `random`
                 exactly as the reference's do (tetris_env.py:187): the global
                 MT19937 state is uploaded before and read back after every
                 call, so a program that seeds `random` gets the reference's
                 games bit-for-bit.  Its GPU work is issued on the stream
                 that was current when it was constructed, with one
                 synchronize per call.
TetrisVecEnv  -- the batched surface: N envs, torch tensors on the GPU,
                 per-env CPython MT19937 streams random.seed(seed + e).
Both run every game rule in the HIP kernels (engine.TetrisBatch); there is no
CPU fallback.
"""
from __future__ import annotations

import collections
import ctypes
import random
import sys
import weakref
from typing import Optional

import numpy as np
import torch

from .. import _lib as C
from .. import spaces
from ..engine import SHAPE_NAMES, TetrisBatch, _mapped, scalar_action


# counter rows of the export record (st_stat)
_TIME, _SCORE, _LINES, _HOLES, _DEATHS, _HEIGHT, _C0, _PIECE = (
    C.STAT[k] for k in ("time", "score", "lines", "holes", "deaths", "piece_height", "count0", "piece"))


def _obs_space(obs_type, width, height, extend_dims):
    """tetris_env.py:381-392."""
    if obs_type == "ram":
        shape = (width, height, 1) if extend_dims else (width, height)
    elif obs_type == "grayscale":
        shape = (84, 84, 1) if extend_dims else (84, 84)
    elif obs_type == "rgb":
        shape = (84, 84, 3)
    else:
        return None
    return spaces.Box(0, 1, shape=shape, dtype=np.float32)


def _stream_sync(sp: ctypes.c_void_p):
    """A synchronize of stream `sp` through libsimpletetris (st_stream_sync:
    the runtime its kernels use; torch's stream synchronize costs ~3 us more
    per call)."""
    fn = C.load().st_stream_sync

    def sync():
        C.check(fn(sp))
    return sync


class TetrisEnv:
    metadata = {"render.modes": ["human", "rgb_array"], "render_fps": 8}  # :339

    def __init__(self, width=10, height=20, obs_type="ram", extend_dims=False,
                 render_mode="rgb_array", reward_step=False, penalise_height=False,
                 penalise_height_increase=False, advanced_clears=False, high_scoring=False,
                 penalise_holes=False, penalise_holes_increase=False, lock_delay=0,
                 step_reset=False, *, device=None, rng: str = "global", seed: Optional[int] = None):
        if rng not in ("global", "private"):
            raise ValueError("rng must be 'global' (CPython's random, like the reference) or 'private'")
        self.width = width
        self.height = height
        self.obs_type = obs_type
        self.extend_dims = extend_dims
        self.render_mode = render_mode
        self.window_size = 512
        self.engine = TetrisBatch(1, width=width, height=height, lock_delay=lock_delay,
                                  step_reset=step_reset, reward_step=reward_step,
                                  penalise_height=penalise_height,
                                  penalise_height_increase=penalise_height_increase,
                                  advanced_clears=advanced_clears, high_scoring=high_scoring,
                                  penalise_holes=penalise_holes,
                                  penalise_holes_increase=penalise_holes_increase,
                                  autoreset="none", device=device,
                                  validate_actions=False)  # step() checks the action itself
        self._rng_mode = rng
        self.engine.seed([0 if seed is None else seed])
        if rng == "global" and seed is not None:
            random.seed(seed)
        self._scoring = dict(advanced_clears=advanced_clears, penalise_height=penalise_height,
                             penalise_height_increase=penalise_height_increase)
        self.action_space = spaces.Discrete(7)           # :377
        self.observation_space = _obs_space(obs_type, width, height, extend_dims)
        self.window = None
        self.clock = None
        self._stats = None         # last downloaded counters (host int64 [NSTAT])
        # info['statistics'] is ONE dict for the env's lifetime, updated in
        # place, like the reference's live shape_counts (tetris_env.py:181,
        # :199, :240): a held info sees later spawns, and counts written into
        # it weight the next draws (:183-191)
        self._shape_counts = None
        self._shape_vals = None    # what the env last wrote into it
        self._started = False
        self._rng_sync_state = None
        dev = self.engine.device
        L = self.engine._L
        # per-step plumbing without per-call allocations: one device tensor per
        # action value, the step's outputs, and ONE read-back record
        # (st_export_env: obs words | reward | done | counters | MT words in
        # 'global' mode | float32 obs for 'ram') plus the image for grayscale /
        # rgb, copied into pinned host buffers and waited for once
        self._acts = [torch.full((1,), a, dtype=torch.uint8, device=dev) for a in range(7)]
        self._p_acts = [ctypes.c_void_p(t.data_ptr()) for t in self._acts]
        self._nrec = int(L.st_export_words(width, height))
        self._parts = (C.EXPORT_MT if rng == "global" else 0) | (C.EXPORT_OBS_F32 if obs_type == "ram" else 0)
        self._f32_at = width + 2 + C.NSTAT + C.MT_N  # the record's float32 obs
        self._d_rec = torch.empty(self._nrec, dtype=torch.int32, device=dev)
        self._h_rec = torch.empty(self._nrec, dtype=torch.int32, pin_memory=True)
        self._h_rec_np = self._h_rec.numpy()
        self._zeros = torch.zeros((width, 1), dtype=torch.int32, device=dev)
        self._ch = 1 if obs_type == "grayscale" else 3
        if obs_type in ("grayscale", "rgb"):
            self._d_img = torch.empty((1, 84, 84, self._ch), dtype=torch.float32, device=dev)
            self._h_img = torch.empty((1, 84, 84, self._ch), dtype=torch.float32, pin_memory=True)
        self._h_mt = np.zeros(C.MT_N, np.uint32)
        self._h_idx = np.zeros(1, np.int32)
        # the export and image kernels write straight into the pinned buffers
        # when the runtime maps them for the device (else: device buffer + copy)
        self._rec_dst = _mapped(self._h_rec)
        self._img_dst = _mapped(self._h_img) if obs_type in ("grayscale", "rgb") else None
        # per-step constants: output pointers, the stream current at
        # construction (the env issues all its work there), a direct
        # hipStreamSynchronize (torch's costs ~3 us more per call)
        self._po, self._pr, self._pd = (ctypes.c_void_p(t.data_ptr())
                                        for t in (self.engine.obs, self.engine.reward, self.engine.done))
        self._pz = ctypes.c_void_p(self._zeros.data_ptr())
        self._sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        self._sync = _stream_sync(self._sp)

    # ------------------------------------------------------------- RNG mirror
    def seed(self, seed=None):
        """Seed the piece RNG: random.seed(seed) in 'global' mode (what a user
        of the reference does), the env's private MT19937 otherwise."""
        if self._rng_mode == "global":
            random.seed(seed)
        else:
            self.engine.seed([0 if seed is None else seed])
        return [seed]

    def _stream(self):
        return self._sp

    def _push_rng(self):
        if self._rng_mode != "global":
            return
        state = random.getstate()
        if self._rng_sync_state is not None and state == self._rng_sync_state:
            return
        internal = state[1]
        self._h_mt[:] = np.asarray(internal[:C.MT_N], dtype=np.uint32)
        self._h_idx[0] = internal[C.MT_N]
        v = self.engine._views
        L = self.engine._L
        s = self._stream()
        C.check(L.st_copy(ctypes.c_void_p(v.mt), ctypes.c_void_p(self._h_mt.ctypes.data),
                          C.MT_N * 4, s))
        C.check(L.st_copy(ctypes.c_void_p(v.stats + C.STAT["mt_index"] * v.stride * 4),
                          ctypes.c_void_p(self._h_idx.ctypes.data), 4, s))
        self._rng_sync_state = state  # the device now mirrors CPython's state

    def _readback(self, obs_ptr, rew_ptr, done_ptr, prev_idx=None):
        """One read-back per call: the env's record (st_export_env: outputs,
        counters, CPython's form of its MT state in 'global' mode and the
        float32 obs for 'ram') and, for image observations, its image, each
        written to pinned host memory on the stream, then ONE synchronize.
        In 'global' mode CPython's random takes the env's MT state if this
        call drew pieces.  Returns (float32 obs [W, H] for 'ram' else None,
        reward, done, counters [NSTAT] as Python ints, image or None)."""
        eng = self.engine
        L, ctx = eng._L, eng._ctx
        s = self._stream()
        if self._rec_dst is not None:
            C.check(L.st_export_env(ctx, 0, obs_ptr, rew_ptr, done_ptr, self._parts, self._rec_dst, s))
        else:
            C.check(L.st_export_env(ctx, 0, obs_ptr, rew_ptr, done_ptr, self._parts,
                                    ctypes.c_void_p(self._d_rec.data_ptr()), s))
            C.check(L.st_copy(ctypes.c_void_p(self._h_rec.data_ptr()), ctypes.c_void_p(self._d_rec.data_ptr()),
                              self._nrec * 4, s))
        img = None
        if self.obs_type in ("grayscale", "rgb"):
            src = obs_ptr if obs_ptr is not None else ctypes.c_void_p(self._zeros.data_ptr())
            if self._img_dst is not None:
                C.check(L.st_grayscale(ctx, src, 84, self._ch, 0, self._img_dst, s))
            else:
                C.check(L.st_grayscale(ctx, src, 84, self._ch, 0, ctypes.c_void_p(self._d_img.data_ptr()), s))
                C.check(L.st_copy(ctypes.c_void_p(self._h_img.data_ptr()), ctypes.c_void_p(self._d_img.data_ptr()),
                                  self._d_img.numel() * 4, s))
        self._sync()
        rec = self._h_rec_np
        W = self.width
        obs = None
        if self.obs_type == "ram":  # decoded on the device; a fresh array per step, like np.array(state)
            a = self._f32_at
            obs = rec[a:a + W * self.height].view(np.float32).reshape(W, self.height).copy()
        st = rec[W + 2: W + 2 + C.NSTAT].tolist()  # Python ints (the reference's counters are ints)
        if self._rng_mode == "global":
            idx = st[C.STAT["mt_index"]]
            # the cached state is CPython's current one (_push_rng checked it
            # before the step); only a step that drew changes it
            if prev_idx is None or idx != prev_idx or self._rng_sync_state is None:
                mt = rec[W + 2 + C.NSTAT:W + 2 + C.NSTAT + C.MT_N].view(np.uint32)
                old = self._rng_sync_state if self._rng_sync_state is not None else random.getstate()
                new = (old[0], tuple(mt.tolist()) + (idx,), old[2])
                random.setstate(new)
                self._rng_sync_state = new
        if img is None and self.obs_type in ("grayscale", "rgb"):
            img = self._h_img.numpy()[0].copy()
        return obs, int(rec[W]), bool(rec[W + 1]), st, img

    # ------------------------------------------------------------- gym API
    def _get_info(self, st):
        """TetrisEngine.get_info (tetris_env.py:232-241); `st` holds Python
        ints (the record's counter rows, .tolist()).  'statistics' is the
        env's one shape-count dict, refreshed in place (the reference returns
        its live shape_counts, :240)."""
        vals = tuple(st[_C0:_C0 + 7])
        d = self._shape_counts
        if d is None:
            d = self._shape_counts = dict(zip(SHAPE_NAMES, vals))
        elif vals != self._shape_vals:
            for k, v in zip(SHAPE_NAMES, vals):
                d[k] = v
        self._shape_vals = vals
        return {"time": st[_TIME],
                "current_piece": SHAPE_NAMES[st[_PIECE] & 7],
                "score": st[_SCORE],
                "lines_cleared": st[_LINES],
                "holes": st[_HOLES],
                "deaths": st[_DEATHS],
                "statistics": d}

    def _push_counts(self):
        """Counts the caller wrote into info['statistics'] since the last call
        take effect like writes into the reference's shape_counts: the next
        draw (:183-191) sees them, and spawns count on from them (:199).  The
        device drops its preview (st_mt_sync: the piece drawn one spawn ahead
        with the old counts) and takes the new counts."""
        d = self._shape_counts
        if d is None:
            return
        if len(d) == 7 and all(type(d.get(k)) is int for k in SHAPE_NAMES):
            vals = tuple(d[k] for k in SHAPE_NAMES)
            if vals == self._shape_vals:
                return
        else:
            vals = None
        if vals is None or not all(-(1 << 31) <= v < (1 << 31) for v in vals):
            raise ValueError("info['statistics'] may only hold int32 counts for the keys "
                             f"{SHAPE_NAMES} (got {dict(d)!r})")
        eng = self.engine
        L, s, v = eng._L, self._stream(), eng._views
        C.check(L.st_mt_sync(eng._ctx, s))
        cnt = np.asarray(vals, dtype=np.int32)
        for i in range(7):
            C.check(L.st_copy(ctypes.c_void_p(v.stats + (C.STAT["count0"] + i) * v.stride * 4),
                              ctypes.c_void_p(cnt.ctypes.data + 4 * i), 4, s))
        self._sync()  # (cnt is pageable host memory)
        self._shape_vals = vals
        if self._stats is not None:
            self._stats[_C0:_C0 + 7] = list(vals)  # the reward-type test compares with these

    def _observation(self, obs, img):
        """TetrisEnv._observation (tetris_env.py:413-433) + float32 cast, from
        the read-back's float32 obs (ram) or image (grayscale / rgb)."""
        if self.obs_type == "ram":
            return obs.reshape(self.width, self.height, 1) if self.extend_dims else obs
        if self.obs_type == "grayscale":
            return img if self.extend_dims else img.reshape(84, 84)
        return img

    def _typed_reward(self, r: int, done: bool, prev, st):
        """Reproduce the Python type the reference's reward ends up with (R18)."""
        if done:
            return int(r)
        if st[_C0:_C0 + 7] == prev[_C0:_C0 + 7]:  # no new piece: the step did not lock
            return int(r)
        if self._scoring["advanced_clears"]:
            hp = _HEIGHT
            if self._scoring["penalise_height"] or (
                    self._scoring["penalise_height_increase"] and st[hp] > prev[hp]):
                return np.float64(r)
            return float(r)
        return np.int64(r)

    def step(self, action):
        """TetrisEnv.step (tetris_env.py:397-403)."""
        if not self._started:
            raise AttributeError("step() before reset(): the reference fails at tetris_env.py:244")
        action = scalar_action(action)  # value_action_map[action]'s KeyError, tetris_env.py:245
        self._push_counts()
        prev = self._stats
        self._push_rng()
        eng = self.engine
        C.check(eng._L.st_step(eng._ctx, self._p_acts[action], self._po, self._pr, self._pd, self._sp))
        obs, r, d, st, img = self._readback(self._po, self._pr, self._pd, prev[C.STAT["mt_index"]])
        self._stats = st
        return self._observation(obs, img), self._typed_reward(r, d, prev, st), d, self._get_info(st)

    def reset(self, return_info=False):
        """TetrisEnv.reset (tetris_env.py:405-411): clear(); obs is the empty
        board (clear() returns the board before the new piece is drawn)."""
        self._push_counts()
        self._push_rng()
        C.check(self.engine._L.st_reset(self.engine._ctx, None, self._sp))  # clear() on the env's stream
        self._started = True
        obs, _, _, st, img = self._readback(self._pz, None, None)
        self._stats = st
        obs = self._observation(obs, img)
        return (obs, self._get_info(st)) if return_info else obs

    def render(self, mode="human"):
        """render('rgb_array'): 160x160x3 uint8 frame (tetris_env.py:458-462)."""
        if mode == "rgb_array":
            self._sync()  # the env's own stream first (its steps), then the current one
            packed = self.engine.render_packed()
            img = self.engine.grayscale(packed, 160, 3, as_u8=True)[0]
            return img.cpu().numpy()
        if mode == "human":
            raise NotImplementedError("render('human') needs pygame; out of scope for the GPU engine")
        raise NotImplementedError(mode)

    def close(self):
        """tetris_env.py:466-467."""
        if getattr(self, "engine", None) is not None:
            self.engine.close()
            self.engine = None


class _SlotLayout:
    """The part sizes and byte offsets of a vector env's output slot,
    computed once per env (every slot of it has the same layout)."""

    def __init__(self, n, width, height, f32, final):
        nd = (n + 3) // 4  # int32 words holding done's n bytes
        wn = width * n
        # whole rows first: obs and the final obs start 16-B aligned whenever
        # n % 4 == 0 (the step kernel's 16-B store path)
        self.sizes = (wn, wn, C.NSTAT * n, n, nd) if final else (wn, C.NSTAT * n, n, nd)
        self.total = sum(self.sizes)
        offs = [0]
        for z in self.sizes[:-1]:
            offs.append(offs[-1] + 4 * z)
        self.offs = tuple(offs)
        self.n, self.width, self.height, self.f32, self.final = n, width, height, f32, final


class _Slot:
    """One set of st_step_vec outputs: with copy=False the vector env
    alternates two; with copy=True every step gets a fresh one, handed to
    the caller (the env never writes it again).  The int32 outputs are views
    of ONE allocation (obs | final obs | info rows | reward | done bytes),
    the float32 obs a second one: two caching-allocator calls per step.  The
    per-step cost of copy=True is these Python-level tensor ops, so only the
    returned obs / reward / done are viewed here; the info rows and the
    final obs are viewed when an info is read (VecInfo)."""

    def __init__(self, lay: _SlotLayout, dev):
        n = lay.n
        self.lay = lay
        flat = torch.empty(lay.total, dtype=torch.int32, device=dev)
        self.parts = parts = flat.split(lay.sizes)  # one op for every part
        self.obs = parts[0].view(lay.width, n)
        self.reward = parts[-2]
        self.done = parts[-1].view(torch.uint8)[:n].view(torch.bool)
        self.obs_f32 = torch.empty((n, lay.width, lay.height), dtype=torch.float32, device=dev) if lay.f32 else None
        base, o = flat.data_ptr(), lay.offs
        vp = ctypes.c_void_p
        self.ptrs = (vp(base), None if self.obs_f32 is None else vp(self.obs_f32.data_ptr()), vp(base + o[-2]),
                     vp(base + o[-1]), vp(base + o[1]) if lay.final else None, vp(base + o[-3]))
        self.owner = None  # weakref to the VecInfo that reads this slot
        self.stream = -1    # the stream its last step was written on (a raw handle value; None =
                            # the null stream; -1 = never written)
        self.busy = 0       # copy=True pool: times it was found held since its last step
        # the root tensor is kept: under torch.inference_mode() views do not
        # keep their base alive, and the baseline below must count only
        # long-lived owners
        self._flat = flat
        self._flat_st = flat.untyped_storage()
        self._f32_st = self.obs_f32.untyped_storage() if self.obs_f32 is not None else None
        self._flat_cd = self._flat_st._cdata
        self._idle = self._refs()  # the counts while only the slot holds its tensors

    def _refs(self):
        """Python references to the tensors step() hands out, and the owners
        of the two allocations (every view of them, the caller's included)."""
        g, use = sys.getrefcount, torch._C._storage_Use_Count
        if self.obs_f32 is None:  # (None's own count moves all the time: not counted)
            return g(self.obs), g(self.reward), g(self.done), use(self._flat_cd)
        return (g(self.obs), g(self.reward), g(self.done), g(self.obs_f32), use(self._flat_cd),
                use(self._f32_st._cdata))

    def idle(self) -> bool:
        """Nothing outside the slot still holds its outputs (no returned
        tensor, view of one, info or info tensor): a copy=True env may write
        the next step into it without touching anything the caller kept."""
        return self._refs() == self._idle

    def info_rows(self):
        return self.parts[-3].view(C.NSTAT, self.lay.n)

    def final_obs(self):
        return self.parts[1].view(self.lay.width, self.lay.n) if self.lay.final else None


class _SlotPool:
    """copy=True's output slots, oldest first.  take() reuses one of the two
    oldest if nothing outside the pool holds it (_Slot.idle) -- callers
    release in order, so a loop that keeps the last d steps' outputs settles
    at d + 1 slots and then allocates nothing -- else builds a new one (the
    oldest is dropped at `cap`).  A slot found held at the front more often
    than the pool is long is kept for good: the pool forgets it (it is freed
    when the caller drops it), so a few kept-forever steps do not block the
    reuse behind them."""

    def __init__(self, cap: int):
        self.q: collections.deque = collections.deque()
        self.cap = cap

    def __len__(self):
        return len(self.q)

    def clear(self):
        self.q.clear()

    def take(self, new):
        """(slot, reused): a released slot, or new() when none is."""
        q = self.q
        if q:  # the common case: the oldest slot was released -- it goes to the back
            z = q[0]
            if z.idle():
                q.rotate(-1)
                z.busy = 0
                return z, True
        return self._take_slow(new)

    def _take_slow(self, new):
        q = self.q
        slot = None
        for i in range(min(2, len(q))):
            z = q[i]
            if z.idle():
                del q[i]
                slot = z
                break
            z.busy += 1
        reused = slot is not None
        if slot is None:
            slot = new()
            if len(q) >= self.cap:
                q.popleft()  # still the caller's: it is freed when they drop it
        while q and q[0].busy > max(8, len(q)) and not q[0].idle():
            q.popleft()
        slot.busy = 0
        q.append(slot)
        return slot, reused


class VecInfo:
    """get_info() (tetris_env.py:232-241) of one TetrisVecEnv step for all N
    envs, as int32 GPU tensors built on first access: time, score,
    lines_cleared, holes, deaths, piece_height, current_piece (shape id, the
    index into SHAPE_NAMES), statistics [7, N]; ep_time / ep_score /
    ep_lines / ep_holes (the finished episode's counters where the env was
    reset in this step, else 0); and, with the gym reset convention,
    final_observation (the terminal obs of the envs reset in this step, in
    the env's obs format; zeros elsewhere) and _final_observation (bool [N],
    which envs those are).

    The step kernel writes the counters into the slot this info reads, so
    building it costs nothing per step.  With copy=True (the default) the
    slot is the caller's; with copy=False the env reuses a slot two steps
    later and copies it into this object first if this info is still alive
    then (a counter tensor taken out of the info and kept past that is a
    view of the slot: clone it to keep it)."""

    def __init__(self, env: "TetrisVecEnv", slot: _Slot):
        self._env = env
        self._slot = slot  # the info rows / final obs are viewed on first access
        self._info = self._final = None
        self._done = slot.done
        self._cache = None

    def _views(self):
        if self._slot is not None:
            self._info, self._final = self._slot.info_rows(), self._slot.final_obs()
            self._slot = None

    def _detach(self):
        """Own copies of the slot's tensors (the env is about to reuse it;
        stream-ordered before the step that overwrites it).  A dict already
        built from the slot is rebuilt from the copies on the next access
        (its counter tensors were views into the slot)."""
        self._views()
        self._info = self._info.clone()
        self._done = self._done.clone()
        if self._final is not None:
            self._final = self._final.clone()
        self._cache = None

    def _load(self):
        if self._cache is None:
            self._views()
            env = self._env
            d = env.engine.info_tensors(self._info)
            d["current_piece"] = self._info[C.STAT["piece"]] & 7
            if self._final is not None:
                fin = torch.where(self._done.unsqueeze(0), self._final, torch.zeros_like(self._final))
                d["final_observation"] = env._obs(fin, None)
                d["_final_observation"] = self._done.clone()
            self._cache = d
        return self._cache

    def __getitem__(self, k):
        return self._load()[k]

    def get(self, k, default=None):
        return self._load().get(k, default)

    def keys(self):
        return self._load().keys()

    def items(self):
        return self._load().items()

    def __contains__(self, k):
        return k in self._load()

    def __iter__(self):
        return iter(self._load())


class TetrisVecEnv:
    """N SimpleTetris-v0 envs stepped together on one GPU.

    step(actions) -> (obs, reward int32 [N], done bool [N], info)
      obs: float32 [N, W, H] ('ram', '(...,1)' with extend_dims), or
           [N, 84, 84(, 1|3)] for 'grayscale' / 'rgb', or the packed uint32
           [W, N] words with obs_format='packed'.
    With autoreset=True (default) envs that died are reset inside the same
    kernel (TetrisEngine.clear).  autoreset_obs='reset' (default; gym's
    vector-env convention): the returned obs of such an env is
    its RESET obs -- the empty board clear() returns (tetris_env.py:306-315,
    :405-411) -- and its terminal observation (what the reference's step
    returned) is in info['final_observation'] (materialised on first access,
    valid where info['_final_observation']); 'terminal': the returned obs is
    the terminal observation itself (no final_observation key).
    info['ep_score'] / ['ep_lines'] / ['ep_time'] / ['ep_holes'] hold the
    finished episode's counters.  One st_step_vec launch per step writes the
    obs, reward, done, the terminal obs and the info counters.  copy=True
    (default; gym's SyncVectorEnv convention, and the reference's step
    returns a fresh np.copy of the board, tetris_env.py:302): the kernel
    writes them into tensors of their own, which the env never touches
    again while the caller keeps any of them -- obs / reward / done / info,
    a view of one, an info tensor (a slot of a recent step is reused once
    none of that is referenced any more, when torch's allocator would hand
    the memory out again: `slots_reused` counts those steps; the pool
    follows how many steps' outputs the caller keeps).  Outputs read on
    another stream: call record_stream(stream) once, as Tensor.record_stream
    for torch's allocator -- a reused slot is then written only after the
    work queued on that stream.  copy=False: they live in one of two output slots
    that alternate, so they are overwritten two steps later (an info object
    kept longer takes a copy; the obs / reward / done tensors do not) -- the
    fast path, for loops that consume each step's outputs right away.
    reset(return_info=True) returns (obs, info) like the reference's
    reset (:405-411): the post-reset counters (time 0, score 0, the new
    current_piece, the persisting deaths and statistics).
    Actions outside 0..6 raise KeyError like the reference's.  By default
    (`validate_actions='async'`) the step kernel checks the actions it loads
    anyway and sets a sticky flag in mapped host memory: no extra launch and
    no sync; the flagged step has already been applied with the bad action
    acting as idle, and the KeyError comes at the next step() after the flag
    is seen or from check_actions().  `validate_actions=True` is the
    reference's immediate KeyError, before any state changes: actions on the
    GPU are checked by a small kernel the step launch is gated on
    (st_gate_actions: the step changes nothing if an action is bad), and the
    host waits for that check only, with the step already queued behind it;
    `False` does not check (out-of-range values act as idle).  Host (numpy /
    list) actions are always checked up front.
    """

    def __init__(self, num_envs: int, width=10, height=20, obs_type="ram", extend_dims=False,
                 reward_step=False, penalise_height=False, penalise_height_increase=False,
                 advanced_clears=False, high_scoring=False, penalise_holes=False,
                 penalise_holes_increase=False, lock_delay=0, step_reset=False, *,
                 device=None, seed: int = 0, global_offset: int = 0, autoreset: bool = True,
                 autoreset_obs: str = "reset", obs_format: str = "f32", validate_actions="async",
                 copy: bool = True):
        if obs_format not in ("f32", "packed"):
            raise ValueError("obs_format must be 'f32' or 'packed'")
        if autoreset_obs not in ("reset", "terminal"):
            raise ValueError("autoreset_obs must be 'reset' (gym's convention) or 'terminal'")
        self.num_envs = int(num_envs)
        self.width, self.height = width, height
        self.obs_type, self.extend_dims, self.obs_format = obs_type, extend_dims, obs_format
        self.autoreset, self.autoreset_obs = bool(autoreset), autoreset_obs
        self.engine = TetrisBatch(self.num_envs, width=width, height=height,
                                  lock_delay=lock_delay, step_reset=step_reset,
                                  reward_step=reward_step, penalise_height=penalise_height,
                                  penalise_height_increase=penalise_height_increase,
                                  advanced_clears=advanced_clears, high_scoring=high_scoring,
                                  penalise_holes=penalise_holes,
                                  penalise_holes_increase=penalise_holes_increase,
                                  autoreset="same_step" if autoreset else "none", device=device,
                                  validate_actions=validate_actions)
        self.engine.seed([seed + global_offset + e for e in range(self.num_envs)])
        self.single_action_space = spaces.Discrete(7)
        self.single_observation_space = _obs_space(obs_type, width, height, extend_dims)
        self.device = self.engine.device
        self._want_f32 = obs_format == "f32" and obs_type == "ram"
        fin = self.autoreset and autoreset_obs == "reset"
        self.copy = bool(copy)
        self._fin = fin
        self._lay = _SlotLayout(self.num_envs, width, height, self._want_f32, fin)
        self._slots = [] if self.copy else [_Slot(self._lay, self.device) for _ in range(2)]
        # copy=True: the slots of recent steps, oldest first, reused once the
        # caller holds nothing of them (_Slot.idle).  The pool grows to the
        # caller's holding depth (a loop that keeps each step's outputs for d
        # steps settles at d + 1 slots, and every step then reuses the oldest:
        # one idle() test per step), up to _SLOT_BYTES of slots
        slot_bytes = 4 * self._lay.total + (4 * self.num_envs * width * height if self._want_f32 else 0)
        self._pool = _SlotPool(max(4, min(64, self._SLOT_BYTES // max(slot_bytes, 1))))
        self.slots_reused = 0
        self._consumers: list = []  # record_stream: streams that read the outputs
        self._k = 0
        self._step_vec = self.engine._L.st_step_vec
        self._stream_wait = self.engine._L.st_stream_wait

    _SLOT_BYTES = 1 << 30  # copy=True: most memory the slot pool keeps for reuse

    def _new_slot(self):
        return _Slot(self._lay, self.device)

    def record_stream(self, stream) -> None:
        """Declare that the outputs of this env's steps are read on `stream`
        (a torch.cuda.Stream or a raw hipStream_t handle) -- the vector env's
        counterpart of Tensor.record_stream, which torch's caching allocator
        honours and this env's output slots do as well: before a step writes
        into a slot again (a copy=True slot the caller released, or
        copy=False's alternating slots), the env's stream waits, on the
        device, for the work queued on every registered stream by then.  A
        consumer on the env's own stream needs nothing (stream order)."""
        h = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
        if all(c.value != h for c in self._consumers):
            self._consumers.append(ctypes.c_void_p(h))

    def _order_reuse(self, s: ctypes.c_void_p, prev) -> None:
        """A slot is written on stream s again: s waits for the registered
        consumer streams and for the stream that last wrote it (if another)."""
        waits = [c for c in self._consumers if c.value != s.value]
        if prev != -1 and prev != s.value:
            waits.append(ctypes.c_void_p(prev))
        if waits:
            with torch.cuda.device(self.device):
                for c in waits:
                    C.check(self._stream_wait(s, c))

    def _obs(self, packed, f32):
        if self.obs_format == "packed":
            return packed
        if self.obs_type == "ram":
            o = f32 if f32 is not None else self.engine.obs_to_f32(packed)
            return o.unsqueeze(-1) if self.extend_dims else o
        ch = 1 if self.obs_type == "grayscale" else 3
        g = self.engine.grayscale(packed, 84, ch)
        return g if (self.obs_type == "rgb" or self.extend_dims) else g.squeeze(-1)

    def reset(self, return_info: bool = False):
        """TetrisEnv.reset (tetris_env.py:405-411) for every env: clear()
        (:306-315), whose observation is the empty board; with return_info
        also get_info() after the reset (:232-241) as a dict of [N] tensors
        (ep_* 0: no episode finished in a reset)."""
        self.engine.reset()
        zeros = torch.zeros((self.width, self.num_envs), dtype=torch.int32, device=self.device)
        if self.obs_format == "packed":
            obs = zeros
        else:
            obs = self._obs(zeros, torch.zeros((self.num_envs, self.width, self.height),
                                               device=self.device) if self.obs_type == "ram" else None)
        if not return_info:
            return obs
        st = self.engine.state_tensors(("stats",), sync=False)["stats"][:, :self.num_envs].clone()
        for k in ("ep_time", "ep_score", "ep_lines", "ep_holes"):
            st[C.STAT[k]] = 0
        info = self.engine.info_tensors(st)
        info["current_piece"] = st[C.STAT["piece"]] & 7
        return obs, info

    def step(self, actions):
        eng = self.engine
        a, gated = eng._actions(actions, gate=True)
        s = eng._stream()
        if self.copy:  # this step's outputs, the caller's from now on
            slot, reused = self._pool.take(self._new_slot)
            if reused:
                self.slots_reused += 1
                if self._consumers or slot.stream != s.value:  # (a reused slot was written before)
                    self._order_reuse(s, slot.stream)
        else:
            slot = self._slots[self._k]
            self._k ^= 1
            held = slot.owner() if slot.owner is not None else None
            if held is not None:  # an info from two steps ago is still alive: it keeps a copy
                held._detach()
            if self._consumers or (slot.stream != -1 and slot.stream != s.value):
                self._order_reuse(s, slot.stream)
        slot.stream = s.value
        po, pf, pr, pd, pfin, pinfo = slot.ptrs
        if gated:  # validate_actions=True, device actions: the step is gated (st_gate_actions)
            eng._gate_launch(a, s)
        try:
            C.check(self._step_vec(eng._ctx, ctypes.c_void_p(a.data_ptr()), po, pf, pr, pd, pfin, pinfo, s))
        except BaseException:
            if gated:
                eng._gate_abort()
            raise
        if gated:
            eng._gate_wait()  # waits for the check only; raises KeyError if the step was skipped
        info = VecInfo(self, slot)
        if not self.copy:
            slot.owner = weakref.ref(info)
        return self._obs(slot.obs, slot.obs_f32), slot.reward, slot.done, info

    def check_actions(self):
        """validate_actions='async': raise KeyError if an action outside 0..6
        reached any step so far (waits for the queued work)."""
        self.engine.check_actions()

    def close(self):
        self._pool.clear()
        self.engine.close()
