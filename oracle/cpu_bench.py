"""CPU baseline worker for bench.py's cpu_baseline leg (TEST INFRASTRUCTURE:
the C oracle is the thing timed here as the reported CPU baseline, never the
product path).

    python -m oracle.cpu_bench --envs 4096 --offset 0 --seconds 10 [--config c4]

Runs the oracle (a restatement of TetrisEngine.step, tetris_env.py:243-304)
over `envs` envs with seeds 1000 + global index and the bench's splitmix64
action stream, auto-resetting dead envs like the bench, for about `seconds`
seconds of wall time, and prints one JSON line {"env_steps", "seconds"}.
bench.py starts one such process per host core for the all-cores aggregate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import oracle as O  # noqa: E402

CONFIGS = {
    "c3": dict(),
    "c4": dict(advanced_clears=True, penalise_holes_increase=True, penalise_height_increase=True),
}


def run(envs: int, offset: int, seconds: float, config: str = "c3", seed_a: int = 0x5EED,
        chunk: int = 64) -> dict:
    ob = O.OracleBatch(envs, [1000 + offset + e for e in range(envs)], width=10, height=20,
                       **CONFIGS[config])
    ob.reset()
    steps = 0
    t0 = time.perf_counter()
    while True:
        acts = O.splitmix64_actions(seed_a, steps, chunk, envs, offset=offset)
        ob.rollout(acts, want_obs=True, want_stats=False)
        steps += chunk
        if time.perf_counter() - t0 >= seconds:
            break
    return {"env_steps": envs * steps, "seconds": time.perf_counter() - t0, "steps": steps,
            "envs": envs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--offset", type=int, default=0)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    a = ap.parse_args()
    print(json.dumps(run(a.envs, a.offset, a.seconds, a.config)), flush=True)


if __name__ == "__main__":
    main()
