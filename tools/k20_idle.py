"""Does the GPU's idle time before a K = 20 region change the region's
time?  65,536 envs (C3), st_step eager launches; before each region the GPU
is kept busy with st_step launches up to the region's synchronize, then
left idle for `gap` (host sleep) before the region starts.  Prints the
region's wall and event time per step for each gap."""
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
from gym_simpletetris_amd import _lib as C  # noqa: E402

n, K = 65536, 20
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], validate_actions=False)
b.reset()
acts = torch.stack([b.gen_actions(t, 0x5EED).clone() for t in range(64)])
s = torch.cuda.Stream()
sp = ctypes.c_void_p(s.cuda_stream)
L, ctx = b._L, b._ctx
po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
args = [(ctx, ctypes.c_void_p(acts[t].data_ptr()), po, pr, pd, sp) for t in range(64)]
fn = L.st_step
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(s):
    e0.record(s)
    e1.record(s)
torch.cuda.synchronize()
res = {}
for gap_us in (0, 20, 100, 1000, 10000, 100000):
    ws, es = [], []
    for rep in range(12):
        with torch.cuda.stream(s):
            for a in args[:40]:  # busy GPU right up to the synchronize
                fn(*a)
            torch.cuda.synchronize()
            if gap_us:
                t_end = time.perf_counter() + gap_us * 1e-6
                while time.perf_counter() < t_end:
                    pass
            t0 = time.perf_counter()
            e0.record(s)
            for a in args[:K]:
                fn(*a)
            e1.record(s)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
        ws.append((t1 - t0) / K * 1e6)
        es.append(e0.elapsed_time(e1) * 1e3 / K)
    ws.sort()
    es.sort()
    res[gap_us] = {"wall_us_median": ws[len(ws) // 2], "event_us_median": es[len(es) // 2],
                   "wall_us_min": ws[0], "event_us_min": es[0]}
print(json.dumps(res))
