"""Round 5 diagnostic: host cost of one st_step call (ctypes + the C ABI +
hipLaunchKernel) against the kernel's period.  Times, on a warm engine of
65,536 envs: (1) N ctypes calls of a no-compute export (st_wire_words), (2)
N st_step calls enqueued back to back (host time of the loop, and the GPU's
event span), (3) the same with the GPU blocked behind a long first launch
(host submission alone, no queue back-pressure)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

n = 65536
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
eng = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
L, ctx = eng._L, eng._ctx
T = 2200
acts = torch.empty((T, n), dtype=torch.uint8, device=dev)
for t in range(T):
    eng.gen_actions(t, 0x5EED, out=acts[t])
eng.reset()
obs = torch.empty((10, n), dtype=torch.int32, device=dev)
rew = torch.empty(n, dtype=torch.int32, device=dev)
done = torch.empty(n, dtype=torch.uint8, device=dev)
po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (obs, rew, done))
ap = [ctypes.c_void_p(acts[t].data_ptr()) for t in range(T)]
fn = L.st_step
torch.cuda.synchronize()

N = 20000
t0 = time.perf_counter()
for _ in range(N):
    L.st_wire_words(10, 20)
noop = (time.perf_counter() - t0) / N * 1e6
print("ctypes no-op export: %.2f us/call" % noop)

e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(s):
    for t in range(100):
        fn(ctx, ap[t], po, pr, pd, sp)
    torch.cuda.synchronize()
    for K in (20, 200, 2000):
        res = []
        for rep in range(3):
            torch.cuda.synchronize()
            e0.record(s)
            t0 = time.perf_counter()
            for t in range(K):
                fn(ctx, ap[t], po, pr, pd, sp)
            t1 = time.perf_counter()
            e1.record(s)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res.append("host %.2f us/call, gpu %.2f us/step, wall %.2f us/step" % (
                (t1 - t0) / K * 1e6, e0.elapsed_time(e1) * 1e3 / K, (t2 - t0) / K * 1e6))
        print("K=%d: %s" % (K, " | ".join(res)), flush=True)
    # host submission with the GPU busy behind a 200-launch backlog (no idle-queue effects)
    torch.cuda.synchronize()
    for t in range(200):
        fn(ctx, ap[t], po, pr, pd, sp)
    t0 = time.perf_counter()
    for t in range(200, 220):
        fn(ctx, ap[t], po, pr, pd, sp)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print("20 calls behind a backlog: host %.2f us/call" % ((t1 - t0) / 20 * 1e6))
eng.close()
