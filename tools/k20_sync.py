"""K = 20 st_step regions (65,536 envs, C3) bracketed three ways:
  block  -- torch.cuda.synchronize() on both sides (the host thread may sleep
            in it; the region's first launches then issue slowly);
  poll   -- busy-poll the stream until idle (torch.cuda.Stream.query), THEN
            torch.cuda.synchronize() (returns at once), on both sides;
  spin50 -- block, then a 50 us host busy-wait before the region.
Median / min of 15 regions each, wall and HIP-event time per step."""
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


def poll():
    while not s.query():
        pass
    torch.cuda.synchronize()


res = {}
for mode in ("block", "poll", "spin50", "block", "poll", "spin50"):
    ws, es = [], []
    for rep in range(15):
        with torch.cuda.stream(s):
            for a in args[:5]:  # warm-up steps
                fn(*a)
            if mode == "poll":
                poll()
            else:
                torch.cuda.synchronize()
            if mode == "spin50":
                t_end = time.perf_counter() + 50e-6
                while time.perf_counter() < t_end:
                    pass
            t0 = time.perf_counter()
            e0.record(s)
            for a in args[5:5 + K]:
                fn(*a)
            e1.record(s)
            if mode == "poll":
                poll()
            else:
                torch.cuda.synchronize()
            t1 = time.perf_counter()
        ws.append((t1 - t0) / K * 1e6)
        es.append(e0.elapsed_time(e1) * 1e3 / K)
    ws.sort()
    es.sort()
    res.setdefault(mode, []).append({"wall_us_median": round(ws[len(ws) // 2], 3), "event_us_median": round(es[len(es) // 2], 3),
                                     "wall_us_min": round(ws[0], 3)})
print(json.dumps(res))
