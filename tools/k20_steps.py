"""Per-launch GPU time inside a short eager region (the driver's --steps 20):
events between consecutive st_step launches at 65,536 envs, after a
synchronize, repeated; shows whether the first launches after the GPU went
idle run slower than the steady state."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

K, REPS = 20, 6
n = 65536
dev = torch.device("cuda", 0)
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
T = 100 + REPS * K * 2
acts = torch.empty((T, n), dtype=torch.uint8, device=dev)
for t in range(T):
    b.gen_actions(t, 0x5EED, out=acts[t])
b.reset()
torch.cuda.synchronize()
L, ctx = b._L, b._ctx
po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
ap = [ctypes.c_void_p(acts[t].data_ptr()) for t in range(T)]
ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
t = 0
with torch.cuda.stream(s):
    for e in ev:
        e.record(s)
    for _ in range(100):
        C.check(L.st_step(ctx, ap[t], po, pr, pd, sp))
        t += 1
    torch.cuda.synchronize()
    for idle_ms in (0.0, 0.0, 1.0, 10.0, 100.0, 0.0):
        time.sleep(idle_ms / 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            ev[i].record(s)
            C.check(L.st_step(ctx, ap[t], po, pr, pd, sp))
            t += 1
        ev[K].record(s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e6
        per = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(K)]
        print(json.dumps({"idle_before_ms": idle_ms, "wall_us": round(wall, 1),
                          "per_launch_us": [round(x, 2) for x in per]}), flush=True)
