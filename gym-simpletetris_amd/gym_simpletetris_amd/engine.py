"""TetrisBatch: N independent SimpleTetris engines resident on one MI355X.

Host mirror of TetrisEngine (/root/reference/gym_simpletetris/envs/tetris_env.py:125-335)
for N envs at once.  All game logic runs in the HIP kernels of
libsimpletetris.so (csrc/st_kernels.hip); this class only owns the context,
the output buffers (torch tensors on the device) and the stream plumbing.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib as C

SHAPE_NAMES = ("T", "J", "L", "Z", "S", "I", "O")  # tetris_env.py:19

# Reference constructor kwargs (TetrisEngine.__init__ / TetrisEnv.__init__).
SCORING_KWARGS = ("reward_step", "penalise_height", "penalise_height_increase",
                  "advanced_clears", "high_scoring", "penalise_holes",
                  "penalise_holes_increase")


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream_ptr(device: torch.device) -> ctypes.c_void_p:
    """torch's current stream on `device` (the raw-handle query costs ~0.2 us
    against ~2 us for building the Stream object; per-step hot path)."""
    if _raw_stream is not None:
        return ctypes.c_void_p(_raw_stream(device.index))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: Optional[torch.Tensor]) -> Optional[ctypes.c_void_p]:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _mapped(t: torch.Tensor):
    """Device address of a pinned host tensor (st_host_device_ptr, i.e.
    hipHostGetDevicePointer in the runtime the kernels use), or None if the
    runtime does not map it for the device."""
    L = C.load()
    dp = ctypes.c_void_p()
    rc = L.st_host_device_ptr(ctypes.c_void_p(t.data_ptr()), ctypes.byref(dp))
    return dp if rc == 0 and dp.value else None


def scalar_action(a) -> int:
    """value_action_map[a] (tetris_env.py:152-160, :245) for one action: ints,
    bools and numpy integers index by value; a float finds a key only when it
    equals one (2.0 -> 2, as in a dict lookup); anything else raises KeyError."""
    if isinstance(a, (bool, np.bool_, int, np.integer)):
        v = int(a)
    elif isinstance(a, (float, np.floating)) and float(a).is_integer():
        v = int(a)
    else:
        raise KeyError(a)
    if not 0 <= v < 7:
        raise KeyError(a)
    return v


def _bad_actions(x: torch.Tensor) -> torch.Tensor:
    """Elementwise "not a key of value_action_map" for an action tensor (the
    same rule as scalar_action: floats must be integral)."""
    if x.dtype == torch.bool:
        return torch.zeros_like(x)
    if x.dtype.is_floating_point:
        return ~((x >= 0) & (x <= 6) & (x == torch.floor(x)))
    if x.dtype == torch.uint8:
        return x > 6
    return (x < 0) | (x > 6)


def _from_dlpack(x):
    """A foreign device array (any DLPack producer: __dlpack__ /
    __dlpack_device__, e.g. a learner's action buffer) as a torch tensor over
    the same memory -- no copy; torch tensors and numpy arrays pass through."""
    if isinstance(x, (torch.Tensor, np.ndarray)) or not hasattr(x, "__dlpack__"):
        return x
    return torch.from_dlpack(x)


class TetrisBatch:
    """Batched engine.  `autoreset`: 'none' (exact reference semantics; the
    caller resets done envs, like `if done: env.reset()`) or 'same_step'
    (clear() runs inside the step kernel for envs that died)."""

    def __init__(self, n_envs: int, width: int = 10, height: int = 20, lock_delay: int = 0,
                 step_reset: bool = False, reward_step: bool = False,
                 penalise_height: bool = False, penalise_height_increase: bool = False,
                 advanced_clears: bool = False, high_scoring: bool = False,
                 penalise_holes: bool = False, penalise_holes_increase: bool = False,
                 autoreset: str = "none", device=None, seeds: Optional[Sequence[int]] = None,
                 validate_actions: bool = True):
        self._L = C.load()
        if not torch.cuda.is_available():
            raise RuntimeError("TetrisBatch needs a ROCm GPU (no CPU fallback by design)")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError(f"device must be a GPU, got {device}")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if autoreset not in C.AUTORESET:
            raise ValueError(f"autoreset must be one of {sorted(C.AUTORESET)}")
        kw = dict(reward_step=reward_step, penalise_height=penalise_height,
                  penalise_height_increase=penalise_height_increase,
                  advanced_clears=advanced_clears, high_scoring=high_scoring,
                  penalise_holes=penalise_holes,
                  penalise_holes_increase=penalise_holes_increase, step_reset=step_reset)
        flags = 0
        for k, v in kw.items():
            if v:
                flags |= C.FLAGS[k]
        self.n = int(n_envs)
        self.width, self.height = int(width), int(height)
        self.lock_delay = int(lock_delay)
        self.flags = flags
        self.kwargs = dict(kw, lock_delay=self.lock_delay, width=self.width, height=self.height)
        self.autoreset = autoreset
        self.device = device
        # step()/rollout() reject actions outside 0..6 like the reference's
        # value_action_map[action] KeyError (tetris_env.py:245).  For a device
        # tensor that check costs one device->host sync per call;
        # validate_actions=False skips it (values >= 7 then act as idle), and
        # 'async' lets the step kernel check the actions it loads anyway (a
        # sticky flag in mapped host memory, st_set_action_flag) without a
        # sync: the KeyError comes at the next step()/rollout() after the flag
        # is seen, or from check_actions().
        if validate_actions not in (True, False, "async"):
            raise ValueError("validate_actions must be True, False or 'async'")
        self.validate_actions = validate_actions
        self._flag_h = self._flag_dev = None
        cfg = C.Config(self.width, self.height, self.lock_delay, flags, C.AUTORESET[autoreset])
        ctx = ctypes.c_void_p()
        with torch.cuda.device(device):
            C.check(self._L.st_create(ctypes.byref(ctx), ctypes.byref(cfg), device.index, self.n))
        self._ctx = ctx
        if validate_actions == "async":
            # the step kernels' own action check (st_set_action_flag) into a
            # sticky word of pinned host memory mapped for the device
            self._flag_h = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._flag_np = self._flag_h.numpy()
            self._flag_dev = _mapped(self._flag_h)
            if self._flag_dev is None:
                raise RuntimeError("validate_actions='async' needs pinned host memory mapped for the device")
            C.check(self._L.st_set_action_flag(ctx, self._flag_dev))
        v = C.StateViews()
        C.check(self._L.st_state(ctx, ctypes.byref(v)))
        self._views = v
        self.stride = int(v.stride)
        W, n = self.width, self.n
        # Reused output buffers (valid until the next step, like a vec-env obs buffer).
        self.obs = torch.zeros((W, n), dtype=torch.int32, device=device)  # packed u32 bits
        self.obs_f32: Optional[torch.Tensor] = None
        self.reward = torch.zeros(n, dtype=torch.int32, device=device)
        self.done = torch.zeros(n, dtype=torch.bool, device=device)
        self._act = torch.zeros(n, dtype=torch.uint8, device=device)
        self._seeded = False
        if seeds is not None:
            self.seed(seeds)

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            self._L.st_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return _stream_ptr(self.device)

    def seed(self, seeds: Sequence[int]):
        """random.seed(seeds[e]) for each env (CPython MT19937 init_by_array)."""
        s = np.asarray([int(x) for x in seeds], dtype=object)
        if len(s) != self.n:
            raise ValueError(f"need {self.n} seeds, got {len(s)}")
        arr = np.empty(self.n, np.uint64)
        for i, x in enumerate(s):
            x = abs(int(x))  # random.seed uses abs() of an int seed
            if x >= 1 << 64:
                raise ValueError("seeds must fit in 64 bits")
            arr[i] = x
        with torch.cuda.device(self.device):
            C.check(self._L.st_seed(self._ctx, ctypes.c_void_p(arr.ctypes.data), self._stream()))
        self._seeded = True

    def _as_dev_u8(self, x, name) -> torch.Tensor:
        x = _from_dlpack(x)
        if isinstance(x, torch.Tensor):
            t = x.to(device=self.device, dtype=torch.uint8)
        else:
            t = torch.as_tensor(np.asarray(x, dtype=np.uint8), device=self.device)
        if t.numel() != self.n:
            raise ValueError(f"{name} must have {self.n} entries, got {t.numel()}")
        return t.contiguous()

    def _actions(self, x, lead=(), gate: bool = False):
        """Actions as a contiguous uint8 device tensor of shape lead + (n,).
        The reference raises KeyError for an action outside value_action_map
        (tetris_env.py:152-160, :245); a uint8 cast would wrap -1 to 255 and
        263 to 7, so values are checked BEFORE it:
          validate_actions=True: immediately.  Host arrays on the host; a
            device tensor, with `gate` (step() / the vector env's step): by
            st_gate_actions -- returned as (tensor, True), and the caller
            gates its step launch on it and calls _gate_wait() after it (the
            step is skipped entirely if an action was bad; the host waits for
            the check kernel only, not the stream); without `gate`
            (rollouts, step_wire) one device->host sync;
          'async': by the step kernel itself (st_set_action_flag: the kernel
            sets a sticky word in mapped host memory when an action is > 6,
            polled here without a sync); non-uint8 tensors get their bad values
            mapped to 255 on the device first, so the kernel sees them;
          False: no check (values > 6 act as idle)."""
        shape = tuple(lead) + (self.n,)
        asyn = self.validate_actions == "async"
        gated = gate and self.validate_actions is True
        if asyn:
            self._raise_flagged()
        if (type(x) is torch.Tensor and x.dtype == torch.uint8 and x.device == self.device
                and x.is_contiguous() and tuple(x.shape) == shape):
            # an RL loop's own device buffer: checked in the step kernel
            # ('async'), by the gate (True), or not at all
            if gated:
                return x, True
            if self.validate_actions is not True:
                return (x, False) if gate else x
        x = _from_dlpack(x)
        if isinstance(x, torch.Tensor):
            if x.is_complex():
                raise TypeError(f"actions must be real numbers, got {x.dtype}")
            if tuple(x.shape) != shape and x.numel() != int(np.prod(shape)):
                raise ValueError(f"actions must have shape {shape}, got {tuple(x.shape)}")
            on_dev = x.device == self.device
            if (self.validate_actions is True and not (gated and on_dev)) or not on_dev:
                bad = _bad_actions(x)
                if bool(bad.any()):
                    v = x[bad].flatten()[0].item()
                    raise KeyError(f"action {v} not in 0..6 (tetris_env.py:245)")
            if x.dtype == torch.uint8 and on_dev:
                t = x
            else:
                t = x.to(device=self.device).to(torch.uint8)
                if asyn or (gated and on_dev):  # keep bad values visible to the kernel's check: a cast
                    # may wrap them into 0..6 (int16 256 -> 0, 2.5 -> 2); the sentinel is set after
                    # the cast, in uint8, so no source dtype has to hold 255 (int8 cannot)
                    t = t.masked_fill_(_bad_actions(x).to(self.device), 255)
            t = t.reshape(shape).contiguous()
            return (t, gated and on_dev) if gate else t
        a = np.asarray(x)
        if a.size != int(np.prod(shape)):
            raise ValueError(f"actions must have shape {shape}, got {a.shape}")
        if a.dtype.kind == "f":
            ok = (a >= 0) & (a <= 6) & (a == np.floor(a))
        elif a.dtype.kind in "iub":
            ok = (a >= 0) & (a <= 6)
        else:
            raise TypeError(f"actions must be numbers, got {a.dtype}")
        if a.size and not ok.all():
            v = a.flat[np.flatnonzero(~ok)[0]]
            raise KeyError(f"action {v} not in 0..6 (tetris_env.py:245)")
        t = torch.as_tensor(a.astype(np.uint8).reshape(shape), device=self.device)
        return (t, False) if gate else t

    def _gate_launch(self, a: torch.Tensor, s) -> None:
        """st_gate_actions: check `a` on stream s; the next step launch on
        this context is skipped if an action is outside 0..6."""
        C.check(self._L.st_gate_actions(self._ctx, _ptr(a), s))

    def _gate_wait(self) -> None:
        """st_gate_wait: wait for the gate's check (not the step behind it)
        and raise the reference's KeyError (tetris_env.py:245) if it saw an
        action outside 0..6 -- the gated step changed nothing."""
        rc = self._L.st_gate_wait(self._ctx)
        if rc < 0:
            C.check(rc)
        if rc:
            raise KeyError("an action outside 0..6 (tetris_env.py:245); no env was stepped")

    def _gate_abort(self) -> None:
        """The gated step's launch failed: end the gate (st_gate_wait also
        disarms it) so that it cannot gate a later step; its answer is moot."""
        self._L.st_gate_wait(self._ctx)

    def _raise_flagged(self):
        if self._flag_np[0]:
            self._flag_np[0] = 0
            raise KeyError("an action outside 0..6 reached an earlier step (validate_actions='async'; "
                           "tetris_env.py:245); it acted as idle")

    def check_actions(self):
        """validate_actions='async': wait for the work queued so far and raise
        KeyError if any checked action was outside 0..6."""
        if self.validate_actions != "async":
            return
        torch.cuda.current_stream(self.device).synchronize()
        self._raise_flagged()

    def reset(self, mask=None):
        """TetrisEngine.clear() on every env (mask None) or where mask != 0."""
        if not self._seeded:
            raise RuntimeError("seed() before reset()")
        m = None if mask is None else self._as_dev_u8(mask, "mask")
        with torch.cuda.device(self.device):
            C.check(self._L.st_reset(self._ctx, _ptr(m), self._stream()))

    def step(self, actions, obs: str = "packed", out=None):
        """One TetrisEngine.step on every env.  obs: 'packed' (u32 [W][n]),
        'f32' (also float32 [n][W][H], fused in the kernel) or 'none'.
        Returns (obs, reward int32 [n], done bool [n]) -- reused buffers, or
        the caller's `out` = (packed obs int32 [W][n], reward int32 [n],
        done uint8/bool [n]) device tensors (e.g. a gather buffer's views)."""
        if obs not in ("packed", "f32", "none"):
            raise ValueError("obs must be 'packed', 'f32' or 'none'")
        a, gated = self._actions(actions, gate=True)
        o_t, r_t, d_t = (self.obs, self.reward, self.done) if out is None else out
        if out is not None:
            for t, dt, shape in ((o_t, torch.int32, (self.width, self.n)),
                                 (r_t, torch.int32, (self.n,)), (d_t, None, (self.n,))):
                if t.device != self.device or tuple(t.shape) != shape or not t.is_contiguous() \
                        or (dt is not None and t.dtype != dt) \
                        or (dt is None and t.dtype not in (torch.uint8, torch.bool)):
                    raise ValueError(f"out tensor {tuple(t.shape)} {t.dtype} on {t.device}: "
                                     f"need contiguous {shape} on {self.device}")
        s = self._stream()
        if gated:  # validate_actions=True, device actions: the gated step (st_gate_actions)
            self._gate_launch(a, s)
        try:
            # no torch.cuda.device() context: st_step selects the context's device itself
            if obs == "f32":
                if self.obs_f32 is None:
                    self.obs_f32 = torch.zeros((self.n, self.width, self.height),
                                               dtype=torch.float32, device=self.device)
                C.check(self._L.st_step_f32(self._ctx, _ptr(a), _ptr(o_t), _ptr(self.obs_f32),
                                            _ptr(r_t), _ptr(d_t), s))
            else:
                C.check(self._L.st_step(self._ctx, _ptr(a), _ptr(o_t) if obs == "packed" else None,
                                        _ptr(r_t), _ptr(d_t), s))
        except BaseException:
            if gated:
                self._gate_abort()
            raise
        if gated:
            self._gate_wait()
        if obs == "f32":
            return self.obs_f32, r_t, d_t
        return (o_t if obs == "packed" else None), r_t, d_t

    @property
    def wire_words(self) -> int:
        """uint32 rows per env of the gather format (st_wire_words)."""
        return C.check_count(self._L.st_wire_words(self.width, self.height))

    def step_wire(self, actions, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One step (as step()) writing BASELINE C5's gather format instead
        of obs / reward / done: int32 [wire_words, n], per env column x's obs
        bits at bit x*H, then the reward's 32 bits and done
        (st_step_wire; `unwire` restores step()'s outputs bit-exactly)."""
        a = self._actions(actions)
        shape = (self.wire_words, self.n)
        if out is None:
            out = torch.empty(shape, dtype=torch.int32, device=self.device)
        elif out.device != self.device or tuple(out.shape) != shape or out.dtype != torch.int32 \
                or not out.is_contiguous():
            raise ValueError(f"out tensor {tuple(out.shape)} {out.dtype} on {out.device}: "
                             f"need contiguous int32 {shape} on {self.device}")
        C.check(self._L.st_step_wire(self._ctx, _ptr(a), _ptr(out), self._stream()))
        return out

    def rollout(self, actions: torch.Tensor, obs: str = "packed", out: Optional[dict] = None):
        """K consecutive steps in one kernel launch (st_rollout).

        actions: uint8 [K, n] on the device.  Returns (obs, reward, done) with
        a leading K dimension: packed obs int32 [K, W, n] ('packed'), float32
        [K, n, W, H] ('f32') or None ('none'); reward int32 [K, n]; done bool
        [K, n].  Identical to K calls of step().  `out` may supply the output
        tensors (keys 'obs', 'obs_f32', 'reward', 'done') to reuse buffers."""
        actions = _from_dlpack(actions)
        if not isinstance(actions, torch.Tensor) or actions.dim() != 2 or actions.shape[1] != self.n \
                or actions.shape[0] < 1:
            raise ValueError(f"actions must be a [K, {self.n}] integer tensor")
        K = int(actions.shape[0])
        actions = self._actions(actions, lead=(K,))
        out = {} if out is None else out
        W, H, n, dev = self.width, self.height, self.n, self.device

        def buf(key, shape, dtype):
            t = out.get(key)
            if t is None or tuple(t.shape) != shape or t.dtype != dtype:
                t = torch.empty(shape, dtype=dtype, device=dev)
                out[key] = t
            return t
        o = buf("obs", (K, W, n), torch.int32) if obs in ("packed", "f32") else None
        f = buf("obs_f32", (K, n, W, H), torch.float32) if obs == "f32" else None
        r = buf("reward", (K, n), torch.int32)
        d = buf("done", (K, n), torch.bool)
        with torch.cuda.device(dev):
            C.check(self._L.st_rollout(self._ctx, K, _ptr(actions), _ptr(o), _ptr(f), _ptr(r),
                                       _ptr(d), self._stream()))
        return (f if obs == "f32" else o), r, d

    def step_n(self, actions: torch.Tensor, obs: str = "packed"):
        """K consecutive steps, one st_step kernel launch each, enqueued by
        ONE library call (st_step_n: the launch loop runs in C, with no
        Python between the launches).  actions: uint8 [K, n] on the device
        (checked like rollout()'s).  Identical to K calls of step(); returns
        the LAST step's (obs, reward, done) in the engine's reused buffers
        ('packed': int32 [W, n], 'f32': float32 [n, W, H], 'none': None)."""
        actions = _from_dlpack(actions)
        if not isinstance(actions, torch.Tensor) or actions.dim() != 2 or actions.shape[1] != self.n \
                or actions.shape[0] < 1:
            raise ValueError(f"actions must be a [K, {self.n}] integer tensor")
        if obs not in ("packed", "f32", "none"):
            raise ValueError("obs: 'packed', 'f32' or 'none'")
        K = int(actions.shape[0])
        actions = self._actions(actions, lead=(K,))
        if obs == "f32" and self.obs_f32 is None:
            self.obs_f32 = torch.zeros((self.n, self.width, self.height), dtype=torch.float32, device=self.device)
        row = actions.stride(0)
        base = actions.data_ptr()
        ptrs = (ctypes.c_void_p * K)(*[base + t * row for t in range(K)])
        C.check(self._L.st_step_n(self._ctx, ctypes.addressof(ptrs), K,
                                  _ptr(self.obs) if obs != "none" else None,
                                  _ptr(self.obs_f32) if obs == "f32" else None,
                                  _ptr(self.reward), _ptr(self.done), self._stream()))
        if obs == "f32":
            return self.obs_f32, self.reward, self.done
        return (self.obs if obs == "packed" else None), self.reward, self.done

    # ------------------------------------------------------------ observations
    def obs_to_f32(self, packed: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Packed obs -> float32 [n][W][H] (the reference's np.float32 board)."""
        packed = self.obs if packed is None else packed
        out = torch.empty((self.n, self.width, self.height), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            C.check(self._L.st_obs_to_f32(self._ctx, _ptr(packed), _ptr(out), self._stream()))
        return out

    def grayscale(self, packed: Optional[torch.Tensor] = None, size: int = 84, channels: int = 1,
                  as_u8: bool = False) -> torch.Tensor:
        """convert_grayscale(board, size) [+ _rgb] per env: [n][size][size][channels]."""
        packed = self.obs if packed is None else packed
        out = torch.empty((self.n, size, size, channels),
                          dtype=torch.uint8 if as_u8 else torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            C.check(self._L.st_grayscale(self._ctx, _ptr(packed), size, channels, int(as_u8),
                                         _ptr(out), self._stream()))
        return out

    # ------------------------------------------------------------ state
    def _sizes(self):
        W, sd = self.width, self.stride
        return dict(board=(W, sd), piece=(sd,), stats=(C.NSTAT, sd), mt=(sd, int(self._views.mt_pitch)))

    def _view_ptr(self, name):
        return getattr(self._views, name)

    def sync_mt(self):
        """Complete the generations the lazy in-kernel MT twist left in
        progress (st_mt_sync): afterwards stats/mt hold CPython's state."""
        if not hasattr(self._L, "st_mt_sync"):  # only an ST_LIB A/B build predating it
            return
        with torch.cuda.device(self.device):
            C.check(self._L.st_mt_sync(self._ctx, self._stream()))

    def state_tensors(self, fields=("board", "piece", "stats"), sync: bool = True) -> dict:
        """Device copies of the state (full stride; slice [..., :n] for real envs).
        `sync=False` skips st_mt_sync: the MT index row then carries engine
        bits (the counters are exact either way)."""
        out = {}
        if sync and ("stats" in fields or "mt" in fields):
            self.sync_mt()
        s = self._stream()
        for f in fields:  # st_copy runs on the stream's device: no device context needed
            shape = self._sizes()[f]
            t = torch.empty(shape, dtype=torch.int32, device=self.device)
            C.check(self._L.st_copy(_ptr(t), ctypes.c_void_p(self._view_ptr(f)), t.numel() * 4, s))
            out[f] = t
        return out

    def get_state(self, fields=("board", "piece", "stats", "mt")) -> dict:
        """Host (numpy, uint32/int32) copy of the state of the real envs."""
        t = self.state_tensors(fields)
        torch.cuda.synchronize(self.device)
        out = {}
        for f, v in t.items():
            a = v.cpu().numpy()
            if f in ("board", "piece", "mt"):
                a = a.view(np.uint32)
            out[f] = a[: self.n, : C.MT_N] if f == "mt" else a[..., : self.n]
        return out

    def set_state(self, **fields):
        """Upload state arrays for the real envs (shapes as returned by
        get_state); padding envs keep their current state."""
        cur = self.state_tensors(tuple(fields))
        # `piece` aliases stats row 14: upload it after `stats`
        order = sorted(fields, key=lambda f: ("stats", "board", "mt", "piece").index(f))
        with torch.cuda.device(self.device):
            for f in order:
                v = fields[f]
                full = cur[f].cpu().numpy().view(np.uint32).copy()
                v = np.asarray(v).astype(np.int64).astype(np.uint32)
                if f == "mt":
                    full[: self.n, : C.MT_N] = v
                else:
                    full[..., : self.n] = v
                t = torch.from_numpy(full.view(np.int32)).to(self.device)
                C.check(self._L.st_copy(ctypes.c_void_p(self._view_ptr(f)), _ptr(t),
                                        t.numel() * 4, self._stream()))
            torch.cuda.synchronize(self.device)

    def save(self, path: Optional[str] = None) -> bytes:
        """Snapshot of every env's state (st_save: board, piece, counters,
        shape counts, MT19937 state); written to `path` if given."""
        nbytes = int(self._L.st_state_bytes(self._ctx))
        buf = ctypes.create_string_buffer(nbytes)
        with torch.cuda.device(self.device):
            C.check(self._L.st_save(self._ctx, ctypes.cast(buf, ctypes.c_void_p), nbytes))
        data = buf.raw
        if path is not None:
            with open(path, "wb") as f:
                f.write(data)
        return data

    def load(self, snapshot) -> None:
        """Restore a snapshot from save() (bytes or a file path) into this
        batch (same width, height and env count)."""
        if isinstance(snapshot, (str, os.PathLike)):
            with open(snapshot, "rb") as f:
                snapshot = f.read()
        data = bytes(snapshot)
        with torch.cuda.device(self.device):
            C.check(self._L.st_load(self._ctx, data, len(data)))

    def render_packed(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """TetrisEngine.render() (tetris_env.py:317-321): board + current piece,
        packed u32 [W][n], without stepping."""
        out = torch.empty((self.width, self.n), dtype=torch.int32, device=self.device) \
            if out is None else out
        with torch.cuda.device(self.device):
            C.check(self._L.st_render(self._ctx, _ptr(out), self._stream()))
        return out

    def info_tensors(self, stats: Optional[torch.Tensor] = None) -> dict:
        """get_info() (tetris_env.py:232-241) for every env as int32 device
        tensors, from the live state or a `stats` snapshot of it."""
        if stats is None:
            stats = self.state_tensors(("stats",), sync=False)["stats"]
        st = stats[:, : self.n]
        return dict(time=st[C.STAT["time"]], score=st[C.STAT["score"]],
                    lines_cleared=st[C.STAT["lines"]], holes=st[C.STAT["holes"]],
                    deaths=st[C.STAT["deaths"]], piece_height=st[C.STAT["piece_height"]],
                    statistics=st[C.STAT["count0"]: C.STAT["count0"] + 7],
                    ep_time=st[C.STAT["ep_time"]], ep_score=st[C.STAT["ep_score"]],
                    ep_lines=st[C.STAT["ep_lines"]], ep_holes=st[C.STAT["ep_holes"]])

    def policy_greedy(self, t: int, seed: int = 0, explore: int = 30,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Greedy placement actions for the current states (st_policy_greedy):
        a clear-heavy workload generator for benchmarks and tests; `explore`
        per mille of the actions are uniform random (splitmix64 keyed by
        seed, t and the env index)."""
        out = self._act if out is None else out
        with torch.cuda.device(self.device):
            C.check(self._L.st_policy_greedy(self._ctx, ctypes.c_uint64(seed), int(t), int(explore),
                                             _ptr(out), self._stream()))
        return out

    def gen_actions(self, t: int, seed: int, global_offset: int = 0,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Synthetic uniform actions splitmix64(seed ^ ((t<<32) ^ e)) % 7 on device."""
        out = self._act if out is None else out
        with torch.cuda.device(self.device):
            C.check(self._L.st_gen_actions(_ptr(out), self.n, int(t), ctypes.c_uint64(seed),
                                           int(global_offset), self._stream()))
        return out


def unwire(wire: torch.Tensor, width: int, height: int):
    """st_unwire: gathered wire rows int32 [words, n] (st_step_wire, one
    shard's or several shards' concatenated along n) on a GPU -> (packed obs
    int32 [width, n], reward int32 [n], done bool [n]), bit-exact with
    step()'s outputs.  Runs on the tensor's device, on torch's current stream."""
    L = C.load()
    words = C.check_count(L.st_wire_words(width, height))
    if not isinstance(wire, torch.Tensor) or wire.device.type != "cuda" or wire.dtype != torch.int32 \
            or wire.dim() != 2 or wire.shape[0] != words or not wire.is_contiguous():
        raise ValueError(f"wire must be a contiguous int32 [{words}, n] GPU tensor")
    n = wire.shape[1]
    obs = torch.empty((width, n), dtype=torch.int32, device=wire.device)
    reward = torch.empty(n, dtype=torch.int32, device=wire.device)
    done = torch.empty(n, dtype=torch.bool, device=wire.device)
    with torch.cuda.device(wire.device):
        C.check(L.st_unwire(width, height, n, _ptr(wire), _ptr(obs), _ptr(reward), _ptr(done),
                            _stream_ptr(wire.device)))
    return obs, reward, done


def unwire_shards(recv: torch.Tensor, width: int, height: int, n_global: int, out=None):
    """st_unwire_shards: a gather's receive buffer int32 [shards, words,
    n_cap] on a GPU (shard r = the contiguous block shard_range(n_global,
    shards, r), its envs at columns 0 .. count_r - 1) -> (packed obs int32
    [width, n_global], reward int32 [n_global], done bool [n_global]) in
    global env order, bit-exact with step()'s outputs, without assembling the
    shards first.  `out`: optional (obs, reward, done) tensors to write.
    Runs on the tensor's device, on torch's current stream."""
    L = C.load()
    words = C.check_count(L.st_wire_words(width, height))
    if not isinstance(recv, torch.Tensor) or recv.device.type != "cuda" or recv.dtype != torch.int32 \
            or recv.dim() != 3 or recv.shape[1] != words or not recv.is_contiguous():
        raise ValueError(f"recv must be a contiguous int32 [shards, {words}, n_cap] GPU tensor")
    shards, _, cap = recv.shape
    if out is None:
        out = (torch.empty((width, n_global), dtype=torch.int32, device=recv.device),
               torch.empty(n_global, dtype=torch.int32, device=recv.device),
               torch.empty(n_global, dtype=torch.bool, device=recv.device))
    else:  # the kernel writes through raw pointers: check every output like recv
        out = tuple(out)
        want = (((width, n_global), (torch.int32,)), ((n_global,), (torch.int32,)),
                ((n_global,), (torch.bool, torch.uint8)))
        if len(out) != 3:
            raise ValueError("out must be (obs, reward, done)")
        for name, t, (shape, dts) in zip(("obs", "reward", "done"), out, want):
            if not isinstance(t, torch.Tensor) or t.device != recv.device or tuple(t.shape) != shape \
                    or t.dtype not in dts or not t.is_contiguous():
                got = (tuple(t.shape), t.dtype, t.device) if isinstance(t, torch.Tensor) else type(t)
                raise ValueError(f"out {name}: need a contiguous {'/'.join(map(str, dts))} {shape} tensor "
                                 f"on {recv.device}, got {got}")
    obs, reward, done = out
    with torch.cuda.device(recv.device):
        C.check(L.st_unwire_shards(width, height, n_global, shards, cap, _ptr(recv), _ptr(obs), _ptr(reward),
                                   _ptr(done), _stream_ptr(recv.device)))
    return obs, reward, done
