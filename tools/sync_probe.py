"""What does the first host call after a device synchronize cost? (K=20 bench overhead)"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
n = 65536
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
b.reset()
acts = torch.zeros((64, n), dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
e1.record(s)
torch.cuda.synchronize()
L, ctx = b._L, b._ctx
po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
ap = ctypes.c_void_p(acts[0].data_ptr())


def t(label, fn, sync=lambda: torch.cuda.synchronize(dev), reps=5):
    out = []
    for _ in range(reps):
        sync()
        a = time.perf_counter()
        fn()
        out.append((time.perf_counter() - a) * 1e6)
    print(f"{label:45s} " + " ".join(f"{x:7.1f}" for x in out), flush=True)


t("record(s) after synchronize(dev)", lambda: e0.record(s))
t("record(s) after synchronize()", lambda: e0.record(s), sync=torch.cuda.synchronize)
t("record(s) after s.synchronize()", lambda: e0.record(s), sync=s.synchronize)
t("record() default stream after sync", lambda: e0.record())
t("with stream(s): pass", lambda: torch.cuda.stream(s).__enter__())
t("st_gen_actions on s after sync", lambda: C.check(L.st_gen_actions(ap, n, 0, ctypes.c_uint64(1), 0, sp)))
t("st_step on s after sync", lambda: C.check(L.st_step(ctx, ap, po, pr, pd, sp)))


def two():
    e0.record(s)
    e1.record(s)


t("two records", two)


def rec_then_step():
    e0.record(s)
    a = time.perf_counter()
    C.check(L.st_step(ctx, ap, po, pr, pd, sp))
    rec_then_step.d = (time.perf_counter() - a) * 1e6


t("record then step (total)", rec_then_step)
print("  step part of last:", rec_then_step.d)
t("sync only", lambda: None)


def spawned():
    st = b.state_tensors(("stats",), sync=False)["stats"][6:13, :n]
    return int(st.to(torch.int64).sum().item())


def sp_sync():
    spawned()
    torch.cuda.synchronize(dev)


t("record(s) after spawned()+sync", lambda: e0.record(s), sync=sp_sync)


def enter_rec():
    with torch.cuda.stream(s):
        e0.record(s)


t("with stream(s): record after spawned()+sync", enter_rec, sync=sp_sync)
t("with stream(s): record after sync", enter_rec)
