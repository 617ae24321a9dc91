"""The driver's K = 20 region (bench.py timed()) replayed step by step, to find
where its first st_step call loses ~20 us of host time (bench.py's
debug.region_probe; tools/first_launch_probe.py does not reproduce it with
a bare synchronize).  Per region: host time of each of the K ctypes calls,
wall time, HIP-event span.  Modes (interleaved, REPS each):
  bench     bench.py's sequence: spawned-count reduction on the stream, two
            event records, synchronize, event record, K launches, event
            record, synchronize
  nosum     without the spawned-count reduction (torch ops) before it
  noev      without the event record right before the first launch
  bare      synchronize, K launches, synchronize (no torch ops, no events)
With PRELUDES=1 the bare region after one operation each: a device
allocation of a new size (hipMalloc), of a cached size, a device->host
read (.item()), a device copy, a torch kernel.  One JSON line per region."""
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

K = 20
REPS = int(os.environ.get("REPS", "5"))
n = 65536
dev = torch.device("cuda", 0)
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
T = 200
acts = torch.empty((T, n), dtype=torch.uint8, device=dev)
for t in range(T):
    b.gen_actions(t, 0x5EED, out=acts[t])
b.reset()
torch.cuda.synchronize()
L, ctx = b._L, b._ctx
po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
args = [(ctx, ctypes.c_void_p(acts[t].data_ptr()), po, pr, pd, sp) for t in range(T)]
fn = L.st_step
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def spawned():
    st = b.state_tensors(("stats",), sync=False)["stats"][C.STAT["count0"]:C.STAT["count0"] + 7, :n]
    return st.to(torch.int64).sum()


scratch = torch.zeros(7, dtype=torch.int64, device=dev)
grow = [1 << 20]


def prelude(mode):
    """Extra preludes (PRELUDES=1): one operation, then the bare region."""
    if mode == "alloc":  # a never-seen size: the caching allocator calls hipMalloc
        grow[0] += 4096
        torch.empty(grow[0], dtype=torch.uint8, device=dev)
    elif mode == "alloc_cached":  # a size freed before: no hipMalloc
        torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    elif mode == "item":  # a device->host read
        scratch[0].item()
    elif mode == "d2d":  # a device copy on the stream
        C.check(L.st_copy(ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(scratch.data_ptr() + 8), 8, sp))
    elif mode == "torch_kernel":  # a torch kernel on the stream
        scratch.add_(1)


def region(mode, t0):
    with torch.cuda.stream(s):
        prelude(mode)
        if mode in ("bench", "noev"):
            spawned()
        if mode != "bare":
            ev0.record(s)
            ev1.record(s)
        torch.cuda.synchronize()
        if mode in ("bench", "nosum"):
            ev0.record(s)
        hs = []
        a = time.perf_counter()
        for i in range(K):
            fn(*args[t0 + i])
            hs.append(time.perf_counter())
        if mode != "bare":
            ev1.record(s)
        torch.cuda.synchronize()
        z = time.perf_counter()
    calls = [round((y - x) * 1e6, 2) for x, y in zip([a] + hs[:-1], hs)]
    span = round(ev0.elapsed_time(ev1) * 1e3, 1) if mode in ("bench", "nosum") else None
    return {"mode": mode, "host_call_us": calls, "wall_us": round((z - a) * 1e6, 1), "event_span_us": span,
            "sync_after_last_us": round((z - hs[-1]) * 1e6, 1)}


with torch.cuda.stream(s):
    ev0.record(s)
    ev1.record(s)
    for t in range(5):
        fn(*args[t])
torch.cuda.synchronize()
t0 = 5
MODES = ("bench", "nosum", "noev", "bare")
if os.environ.get("PRELUDES"):
    MODES = ("bare", "alloc", "alloc_cached", "item", "d2d", "torch_kernel")
for rep in range(REPS):
    for mode in MODES:
        r = region(mode, t0)
        t0 = (t0 + K) % (T - K)
        r["rep"] = rep
        r["kernarg"] = os.environ.get("HIP_FORCE_DEV_KERNARG")
        print(json.dumps(r), flush=True)
