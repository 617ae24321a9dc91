"""Why is the bench's first K = 20 region slower than later ones?
Three engines (65,536 envs, C3) in one process, each: 5 warm-up st_steps,
then 6 K = 20 regions (torch.cuda.synchronize() on both sides) each after 5
more warm-up steps; engine 1 is the process's first GPU work after seeding,
engine 2 is fresh but the GPU has just run engine 1, engine 3 after 3,000
back-to-back steps of engine 2.  Prints wall / event us per step of every
region."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import gym_simpletetris_amd as G  # noqa: E402
G.tune_runtime()
import torch  # noqa: E402

n, K = 65536, 20
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s = torch.cuda.Stream()
sp = ctypes.c_void_p(s.cuda_stream)
with torch.cuda.stream(s):
    e0.record(s)
    e1.record(s)
out = {}


def engine():
    b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], validate_actions=False)
    acts = torch.empty((3200, n), dtype=torch.uint8, device=b.device)
    for t in range(3200):
        b.gen_actions(t, 0x5EED, out=acts[t])
    b.reset()
    torch.cuda.synchronize()
    po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
    args = [(b._ctx, ctypes.c_void_p(acts[t].data_ptr()), po, pr, pd, sp) for t in range(3200)]
    return b, acts, args


for name in ("first", "second", "after_3000"):
    b, acts, args = engine()
    fn = b._L.st_step
    if name == "after_3000":
        with torch.cuda.stream(s):
            for a in args[:3000]:
                fn(*a)
        torch.cuda.synchronize()
    regs = []
    t = 0
    for r in range(6):
        with torch.cuda.stream(s):
            for a in args[t:t + 5]:
                fn(*a)
            t += 5
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(s)
            for a in args[t:t + K]:
                fn(*a)
            t += K
            e1.record(s)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
        regs.append((round((t1 - t0) / K * 1e6, 3), round(e0.elapsed_time(e1) * 1e3 / K, 3)))
    out[name] = regs
    b.close()
    del acts
print(json.dumps(out))
