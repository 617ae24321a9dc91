"""Time the single-env drop-in TetrisEnv.step() (tetris_env.py:397-403 surface)
against the reference's ~30.5 us/step (32,752 steps/s, 1 core).
Uniform random actions, reset on done, like the survey's probe."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
from gym_simpletetris_amd.envs.tetris_env import TetrisEnv  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
out = {}
for obs_type in ("ram", "grayscale"):
    for rng in ("global", "private"):
        env = TetrisEnv(obs_type=obs_type, rng=rng, seed=0)
        random.seed(1)
        acts = [random.randrange(7) for _ in range(steps)]
        env.reset()
        for a in acts[:200]:  # warm-up
            if env.step(a)[2]:
                env.reset()
        t0 = time.perf_counter()
        resets = 0
        for a in acts:
            if env.step(a)[2]:
                env.reset()
                resets += 1
        dt = time.perf_counter() - t0
        out[f"{obs_type}/{rng}"] = {"us_per_step": dt / steps * 1e6, "steps_per_s": steps / dt,
                                    "resets": resets}
        env.close()
print(json.dumps({"single_env_step": out, "reference_us_per_step_build_container": 1e6 / 32752}))
