"""gym_simpletetris_amd -- MI355X-native batched SimpleTetris engine.

Drop-in for gym-simpletetris' step path (reference:
gym_simpletetris/__init__.py:1-6 registers 'SimpleTetris-v0' ->
gym_simpletetris.envs:TetrisEnv).  `make('SimpleTetris-v0', **kwargs)` returns
the single-env reference surface; `make('SimpleTetris-v0', num_envs=N, ...)`
or `make('SimpleTetrisVec-v0', ...)` the batched one.  When gym or gymnasium
is importable the ids are registered there too.
"""
import os as _os

from .engine import SHAPE_NAMES, TetrisBatch  # noqa: F401
from .envs import TetrisEnv, TetrisVecEnv  # noqa: F401

__version__ = "0.1.0"

ENV_IDS = ("SimpleTetris-v0", "SimpleTetrisVec-v0")


def tune_runtime(force_dev_kernarg: bool = True) -> bool:
    """Opt-in HIP runtime setting for step-per-launch loops: kernel arguments
    in device memory for every launch (HIP_FORCE_DEV_KERNARG=1), measured
    1-5% faster per st_step on MI355X.  It applies to
    every HIP kernel of the process (and its children) and HIP reads it only
    when its runtime starts, so call this before anything touches the GPU;
    an explicit non-empty setting in the environment wins.  Returns whether
    the variable now holds the requested value.  Importing the package
    changes nothing."""
    want = "1" if force_dev_kernarg else "0"
    if not _os.environ.get("HIP_FORCE_DEV_KERNARG"):
        _os.environ["HIP_FORCE_DEV_KERNARG"] = want
    return _os.environ["HIP_FORCE_DEV_KERNARG"] == want


def make(env_id: str = "SimpleTetris-v0", **kwargs):
    """gym.make equivalent for the two registered ids."""
    if env_id not in ENV_IDS:
        raise KeyError(f"unknown env id {env_id!r}; known: {ENV_IDS}")
    if env_id == "SimpleTetrisVec-v0" or "num_envs" in kwargs:
        return TetrisVecEnv(kwargs.pop("num_envs", 1), **kwargs)
    return TetrisEnv(**kwargs)


def _register():
    for modname in ("gym", "gymnasium"):
        try:  # pragma: no cover - neither is installed in the build image
            mod = __import__(modname)
            mod.envs.registration.register(id="SimpleTetris-v0",
                                           entry_point="gym_simpletetris_amd.envs:TetrisEnv")
        except Exception:  # noqa: BLE001
            pass


_register()
