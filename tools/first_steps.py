"""Per-step kernel time of the first steps after reset (event pair around each
eager st_step launch), 65,536 envs C3: where the driver's --steps 20
--warmup 5 region spends its time.  usage: [ST_LIB=lib.so] python tools/first_steps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

n, T = 65536, 60
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
acts = torch.empty((T, n), dtype=torch.uint8, device=dev)
for t in range(T):
    b.gen_actions(t, 0x5EED, out=acts[t])
b.reset()
torch.cuda.synchronize()
L, ctx = b._L, b._ctx
po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(T + 1)]
with torch.cuda.stream(s):
    for e in ev:
        e.record(s)
torch.cuda.synchronize()
with torch.cuda.stream(s):
    ev[0].record(s)
    for t in range(T):
        C.check(L.st_step(ctx, ctypes.c_void_p(acts[t].data_ptr()), po, pr, pd, sp))
        ev[t + 1].record(s)
torch.cuda.synchronize()
us = [ev[t].elapsed_time(ev[t + 1]) * 1e3 for t in range(T)]
print(os.path.basename(os.environ.get("ST_LIB", "in-tree")),
      " ".join(f"{u:.1f}" for u in us[:30]), "| mean 30-60: %.2f" % (sum(us[30:]) / 30))
