"""Wall time per step of the batched Python surface (TetrisVecEnv.step) at
65,536 envs, actions already on the GPU (an RL loop's shape): packed / float32
obs, with and without the per-step action check (validate_actions)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402

n, T = 65536, int(sys.argv[1]) if len(sys.argv) > 1 else 2000
out = {}
for fmt in ("packed", "f32"):
    for val in (False, "async", True):
        v = G.TetrisVecEnv(n, seed=1000, obs_format=fmt, validate_actions=val)
        v.reset()
        acts = torch.randint(0, 7, (64, n), dtype=torch.uint8, device=v.device)
        for t in range(50):
            v.step(acts[t % 64])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(T):
            v.step(acts[t % 64])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / T
        out[f"{fmt}/validate={val}"] = {"us_per_step": dt * 1e6, "env_steps_per_s": n / dt}
        v.close()
print(json.dumps({"vec_env_step": out, "envs": n, "steps": T}))
