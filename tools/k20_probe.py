"""Where does a short timed region (the driver's --steps 20) lose time?
Times K graph-replayed st_step launches at 65,536 envs several ways."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 65536
dev = torch.device("cuda", 0)
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
acts = torch.empty((200 + 8 * K, n), dtype=torch.uint8, device=dev)
for t in range(acts.shape[0]):
    b.gen_actions(t, 0x5EED, out=acts[t])
b.reset()
torch.cuda.synchronize()
L, ctx = b._L, b._ctx
po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
ap = [ctypes.c_void_p(acts[t].data_ptr()) for t in range(acts.shape[0])]
tcur = [0]


def launch(t):
    C.check(L.st_step(ctx, ap[t], po, pr, pd, sp))


with torch.cuda.stream(s):
    for t in range(100):
        launch(t)
torch.cuda.synchronize()
tcur[0] = 100


def graph(k):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(k):
            launch(tcur[0] + i)
    tcur[0] += k
    torch.cuda.synchronize()
    return g


def region(fn, events=None):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if events:
        events[0].record(s)
    fn()
    if events:
        events[1].record(s)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


res = {}
# 1. fresh graph, first replay, events created inside (round-1 bench)
g = graph(K)


def r1():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        g.replay()
        e1.record(s)
    r1.ev = (e0, e1)


w = region(r1)
res["first_replay_events_inside"] = (w * 1e6 / K, r1.ev[0].elapsed_time(r1.ev[1]) * 1e3 / K)
# 2. second replay of the same graph, pre-created events
ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
w = region(g.replay, ev)
res["second_replay_precreated_events"] = (w * 1e6 / K, ev[0].elapsed_time(ev[1]) * 1e3 / K)
w = region(g.replay, ev)
res["third_replay"] = (w * 1e6 / K, ev[0].elapsed_time(ev[1]) * 1e3 / K)
# 3. fresh graph, first replay, pre-created events
g2 = graph(K)
w = region(g2.replay, ev)
res["fresh_graph_first_replay_precreated"] = (w * 1e6 / K, ev[0].elapsed_time(ev[1]) * 1e3 / K)
# 4. eager launches from Python
base = tcur[0]
tcur[0] += K


def eager():
    for i in range(K):
        launch(base + i)


w = region(eager, ev)
res["eager_python"] = (w * 1e6 / K, ev[0].elapsed_time(ev[1]) * 1e3 / K)
# 5. empty region cost
w = region(lambda: None, ev)
res["empty_region_total_us"] = (w * 1e6, ev[0].elapsed_time(ev[1]) * 1e3)
for k, v in res.items():
    print(f"{k:40s} wall {v[0]:8.2f} us/step   event {v[1]:8.2f} us/step")
