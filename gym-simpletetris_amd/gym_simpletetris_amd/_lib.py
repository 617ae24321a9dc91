"""ctypes binding of libsimpletetris.so (include/simpletetris.h).

There is deliberately no CPU fallback: if the in-tree HIP library is missing
or cannot be loaded, importing the engine raises.  Build it with
`make -C gym-simpletetris_amd/csrc` (or `python -c "import __graft_entry__ as g; g.build()"`).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ST_LIB overrides the library path (a custom or variant build).  A build of
# another ABI version is refused unless ST_AB_OLD_ABI=1 (diagnostic A/Bs of
# older builds only: then missing entry points are tolerated and st_state is
# disabled, with a warning).
LIB_PATH = os.environ.get("ST_LIB") or os.path.join(_HERE, "libsimpletetris.so")

ST_OK, ST_EINVAL, ST_ENOMEM, ST_EHIP, ST_ESTATE = 0, -1, -2, -3, -4
ABI_VERSION = 4  # ST_ABI_VERSION of include/simpletetris.h

# st_flags (include/simpletetris.h) keyed by the reference kwarg names
# (TetrisEngine.__init__, tetris_env.py:126-137).
FLAGS = {
    "reward_step": 1 << 0,
    "penalise_height": 1 << 1,
    "penalise_height_increase": 1 << 2,
    "advanced_clears": 1 << 3,
    "high_scoring": 1 << 4,
    "penalise_holes": 1 << 5,
    "penalise_holes_increase": 1 << 6,
    "step_reset": 1 << 7,
}
AUTORESET = {"none": 0, "same_step": 1}

# st_stat rows
STAT = dict(time=0, score=1, lines=2, holes=3, piece_height=4, deaths=5, count0=6, mt_index=13,
            piece=14, ep_time=15, ep_score=16, ep_lines=17, ep_holes=18)
NSTAT = 19
MT_N = 624
EXPORT_MT, EXPORT_OBS_F32 = 1, 2  # st_export_env parts

EXPORTS = ("st_create", "st_destroy", "st_seed", "st_reset", "st_step", "st_step_f32", "st_step_n", "st_step_vec", "st_rollout",
           "st_wire_words", "st_step_wire", "st_unwire", "st_unwire_shards",
           "st_obs_to_f32", "st_render", "st_grayscale", "st_state", "st_copy", "st_mt_sync", "st_state_bytes", "st_save",
           "st_load", "st_export_env", "st_export_words", "st_check_actions", "st_set_action_flag", "st_gate_actions",
           "st_gate_wait", "st_stream_sync", "st_host_device_ptr", "st_stream_wait", "st_gen_actions", "st_policy_greedy", "st_debug_stamps", "st_last_error", "st_abi_version")


class StError(RuntimeError):
    """A C-ABI call returned a negative st_status."""

    def __init__(self, code, msg):
        super().__init__(f"[st {code}] {msg}")
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("lock_delay", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("autoreset", ctypes.c_int32)]


class StateViews(ctypes.Structure):
    _fields_ = [("board", ctypes.c_void_p), ("piece", ctypes.c_void_p),
                ("stats", ctypes.c_void_p), ("mt", ctypes.c_void_p),
                ("n_envs", ctypes.c_int64), ("stride", ctypes.c_int64),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("mt_pitch", ctypes.c_int64)]


_lib = None


def load(path: str = LIB_PATH):
    """Load the HIP engine library (raises if it is absent: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"libsimpletetris.so not found at {path}; build it with "
            "`make -C gym-simpletetris_amd/csrc` (the engine has no CPU fallback)")
    L = ctypes.CDLL(path)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    u32 = ctypes.c_uint32
    sig = {
        "st_create": ([ctypes.POINTER(vp), ctypes.POINTER(Config), ctypes.c_int, i64], ctypes.c_int),
        "st_destroy": ([vp], ctypes.c_int),
        "st_seed": ([vp, vp, vp], ctypes.c_int),
        "st_reset": ([vp, vp, vp], ctypes.c_int),
        "st_step": ([vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "st_step_f32": ([vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "st_step_n": ([vp, vp, ctypes.c_int64, vp, vp, vp, vp, vp], ctypes.c_int),
        "st_step_vec": ([vp, vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "st_rollout": ([vp, i32, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "st_wire_words": ([i32, i32], ctypes.c_int),
        "st_step_wire": ([vp, vp, vp, vp], ctypes.c_int),
        "st_unwire": ([i32, i32, i64, vp, vp, vp, vp, vp], ctypes.c_int),
        "st_unwire_shards": ([i32, i32, i64, i32, i64, vp, vp, vp, vp, vp], ctypes.c_int),
        "st_obs_to_f32": ([vp, vp, vp, vp], ctypes.c_int),
        "st_render": ([vp, vp, vp], ctypes.c_int),
        "st_grayscale": ([vp, vp, i32, i32, i32, vp, vp], ctypes.c_int),
        "st_state": ([vp, ctypes.POINTER(StateViews)], ctypes.c_int),
        "st_copy": ([vp, vp, i64, vp], ctypes.c_int),
        "st_mt_sync": ([vp, vp], ctypes.c_int),
        "st_state_bytes": ([vp], i64),
        "st_save": ([vp, vp, i64], ctypes.c_int),
        "st_load": ([vp, vp, i64], ctypes.c_int),
        "st_export_env": ([vp, i64, vp, vp, vp, u32, vp, vp], ctypes.c_int),
        "st_export_words": ([i32, i32], ctypes.c_int),
        "st_check_actions": ([vp, i64, vp, vp], ctypes.c_int),
        "st_set_action_flag": ([vp, vp], ctypes.c_int),
        "st_gate_actions": ([vp, vp, vp], ctypes.c_int),
        "st_gate_wait": ([vp], ctypes.c_int),
        "st_stream_sync": ([vp], ctypes.c_int),
        "st_host_device_ptr": ([vp, ctypes.POINTER(vp)], ctypes.c_int),
        "st_stream_wait": ([vp, vp], ctypes.c_int),
        "st_gen_actions": ([vp, i64, i64, u64, i64, vp], ctypes.c_int),
        "st_policy_greedy": ([vp, u64, i64, ctypes.c_uint32, vp, vp], ctypes.c_int),
        "st_debug_stamps": ([vp, vp, i64], ctypes.c_int),
        "st_last_error": ([], ctypes.c_char_p),
        "st_abi_version": ([], ctypes.c_int),
    }
    # ST_AB_OLD_ABI=1: a diagnostic A/B of an older build -- tolerate the
    # entry points it predates (never the default, not even with ST_LIB set)
    ab_override = os.environ.get("ST_AB_OLD_ABI") == "1"
    L.st_abi_version.argtypes = []
    L.st_abi_version.restype = ctypes.c_int
    abi = L.st_abi_version()
    if abi != ABI_VERSION and not ab_override:
        raise ImportError(f"{path}: libsimpletetris ABI {abi} != {ABI_VERSION} (rebuild it, or set "
                          "ST_AB_OLD_ABI=1 for a diagnostic A/B of an older build)")
    for name, (args, res) in sig.items():
        if ab_override and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if abi != ABI_VERSION:
        import warnings
        warnings.warn(f"ST_AB_OLD_ABI=1: {path} has ABI {abi}, this package {ABI_VERSION}; "
                      "st_state disabled (raw ctypes A/Bs only)")
        # the state-view struct may differ across ABIs: an older build
        # serves raw ctypes A/Bs only (views read through the wrong struct
        # size tensors from garbage)
        L.st_state = None
    _lib = L
    return L


def check_count(rc: int) -> int:
    """A non-negative count, or the library's error for a negative code."""
    if rc < 0:
        check(rc)
    return rc


def check(rc: int):
    if rc != ST_OK:
        msg = load().st_last_error()
        raise StError(rc, msg.decode() if msg else "")
    return rc
