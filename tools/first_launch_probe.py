"""Host cost of the first st_step launch after the GPU went idle (round 5,
VERDICT r4 #2): the driver's K = 20 region starts right after a blocking
synchronize, and bench.py's region probe shows its first ctypes st_step call
taking ~10-37 us of host time against ~3 us for the later ones.  This times
single calls (perf_counter around the ctypes call) after different
preludes, at 65,536 envs:
  sync      torch.cuda.synchronize(), then the call
  sleep     synchronize + 1 ms sleep, then the call
  tiny      synchronize, one st_gen_actions launch of 64 actions, then the call
  event     synchronize, an event record on the stream, then the call
  b2b       the call right after another st_step (no synchronize)
and, per prelude, the next 3 calls.  One JSON line per (prelude, repeat)."""
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

n = 65536
dev = torch.device("cuda", 0)
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
T = 4000
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
scratch = torch.empty(64, dtype=torch.uint8, device=dev)
psc = ctypes.c_void_p(scratch.data_ptr())
ev = torch.cuda.Event(enable_timing=True)
fn = L.st_step
t = [0]


def call():
    i = t[0] % T
    t[0] += 1
    a = time.perf_counter()
    fn(ctx, ap[i], po, pr, pd, sp)
    return (time.perf_counter() - a) * 1e6


with torch.cuda.stream(s):
    ev.record(s)
    for _ in range(200):
        call()
    torch.cuda.synchronize()
    noop = []
    for _ in range(200):
        a = time.perf_counter()
        L.st_abi_version()
        noop.append((time.perf_counter() - a) * 1e6)
    print(json.dumps({"noop_ctypes_us_median": sorted(noop)[100]}), flush=True)
    for rep in range(6):
        for pre in ("sync", "sleep", "tiny", "event", "b2b"):
            if pre != "b2b":
                torch.cuda.synchronize()
            if pre == "sleep":
                time.sleep(1e-3)
            elif pre == "tiny":
                C.check(L.st_gen_actions(psc, 64, 0, ctypes.c_uint64(1), 0, sp))
            elif pre == "event":
                ev.record(s)
            else:
                call()
            first = call()
            nxt = [call() for _ in range(3)]
            print(json.dumps({"prelude": pre, "rep": rep, "first_us": round(first, 2),
                              "next_us": [round(x, 2) for x in nxt],
                              "kernarg": os.environ.get("HIP_FORCE_DEV_KERNARG")}), flush=True)
    torch.cuda.synchronize()
