"""Round 5 diagnostic: the bench's rollout line (1.31-1.33 us/step) against
the A/B harness's (1.18-1.21) on the same library.  Times 10 rollout launches
of 100 steps (HIP events, back to back after a warm-up launch) on engines
built and aged the two ways: ShardedTetris (as bench.py's Workload) vs a
plain TetrisBatch (as tools/ab_step.py), after N eager st_steps."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402
from gym_simpletetris_amd.distributed import ShardedTetris  # noqa: E402

n, CH = 65536, 100
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)


def rollout_us(eng, acts, t0):
    L, ctx = eng._L, eng._ctx
    o = torch.empty((CH, 10, n), dtype=torch.int32, device=dev)
    r = torch.empty((CH, n), dtype=torch.int32, device=dev)
    d = torch.empty((CH, n), dtype=torch.uint8, device=dev)
    pp = [ctypes.c_void_p(x.data_ptr()) for x in (o, r, d)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        C.check(L.st_rollout(ctx, CH, ctypes.c_void_p(acts[t0].data_ptr()), pp[0], None, pp[1], pp[2], sp))
        e0.record(s)
        for c in range(10):
            C.check(L.st_rollout(ctx, CH, ctypes.c_void_p(acts[t0 + c * CH].data_ptr()), pp[0], None, pp[1], pp[2], sp))
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (10 * CH)


def age(eng, acts, nsteps, obs, rew, done):
    L, ctx = eng._L, eng._ctx
    po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (obs, rew, done))
    with torch.cuda.stream(s):
        for t in range(nsteps):
            C.check(L.st_step(ctx, ctypes.c_void_p(acts[t].data_ptr()), po, pr, pd, sp))
    torch.cuda.synchronize()


T = 4200
for kind in os.environ.get("KINDS", "sharded plain").split():
    if kind == "sharded":
        sh = ShardedTetris(n, seed=1000, rank=0, world=1, device=dev, autoreset="same_step", width=10, height=20)
        eng = sh.engine
    else:
        eng = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
    acts = torch.empty((T, n), dtype=torch.uint8, device=dev)
    for t in range(T):
        eng.gen_actions(t, 0x5EED, out=acts[t])
    eng.reset()
    obs = torch.empty((10, n), dtype=torch.int32, device=dev)
    rew = torch.empty(n, dtype=torch.int32, device=dev)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    res = []
    done_steps = 0
    for target in (300, 1300, 3000):
        age(eng, acts, target - done_steps, obs, rew, done)
        done_steps = target
        res.append(f"after {target}: {rollout_us(eng, acts, 100):.3f}")
        done_steps += 11 * CH  # the rollouts stepped the envs too
    print(kind, " | ".join(res), flush=True)
    eng.close()
