"""Fast A/B timing of one libsimpletetris.so build (ST_LIB=path): graph-replayed
st_step at 65,536 envs for C3 and C4 (the bench workload) and the packed
rollout, event time per step.  usage: ST_LIB=lib.so python tools/ab_step.py [K]"""
import ctypes
import time
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
WU, n = int(os.environ.get("AB_WU", "300")), 65536
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
res = []
for name, kw in (("c3", {}), ("c4", dict(advanced_clears=True, penalise_holes_increase=True,
                                           penalise_height_increase=True))):
    va = os.environ.get("AB_VALIDATE", "True")
    va = {"True": True, "False": False}.get(va, va)
    b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev,
                      validate_actions=va, **kw)
    acts = torch.empty((WU + K, n), dtype=torch.uint8, device=dev)
    for t in range(WU + K):
        b.gen_actions(t, 0x5EED, out=acts[t])
    b.reset()
    torch.cuda.synchronize()
    L, ctx = b._L, b._ctx
    po, pr, pd = (ctypes.c_void_p(x.data_ptr()) for x in (b.obs, b.reward, b.done))
    ap = [ctypes.c_void_p(acts[t].data_ptr()) for t in range(WU + K)]
    with torch.cuda.stream(s):
        for t in range(WU):
            C.check(L.st_step(ctx, ap[t], po, pr, pd, sp))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for t in range(WU, WU + K):
            C.check(L.st_step(ctx, ap[t], po, pr, pd, sp))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    res.append(f"{name} {e0.elapsed_time(e1) * 1e3 / K:.3f}")
    if name == "c3":
        CH = 100
        o = torch.empty((CH, 10, n), dtype=torch.int32, device=dev)
        r = torch.empty((CH, n), dtype=torch.int32, device=dev)
        d = torch.empty((CH, n), dtype=torch.uint8, device=dev)
        pp = [ctypes.c_void_p(x.data_ptr()) for x in (o, r, d)]
        def spawned():
            st = b.state_tensors(("stats",), sync=True)["stats"]
            return int(st[C.STAT["count0"]:C.STAT["count0"] + 7, :n].to(torch.int64).sum())
        # AB_PRE: what happens between the warm-up launch and the timed ones
        # (diagnostics, round 5).  "plock" reads the counters through
        # state_tensors(sync=True), whose st_mt_sync rewinds every env's
        # MT state to CPython's form: the next ~1,000 steps rebuild the
        # successor generations and redraw previews (+30%) -- a state
        # effect of the read, not of the hardware.
        pre = os.environ.get("AB_PRE", "none")
        if pre == "plockwarm":  # the p_lock read used once before the warm-up launch
            spawned()
            pre = "plock"
        with torch.cuda.stream(s):
            C.check(L.st_rollout(ctx, CH, ap[WU], pp[0], None, pp[1], pp[2], sp))  # what happens between the warm-up launch and the timed ones
        if pre == "torchsum_s":  # the reduction on the launch stream instead of the default one
            scratch = torch.zeros((C.NSTAT, b.stride), dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                int(scratch.sum())
        if pre == "plock_s":  # the p_lock read with every op on the launch stream
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                sp0 = spawned()
            pre = "plock_done"
        if pre in ("copy", "torchsum", "alloc"):
            scratch = torch.zeros((C.NSTAT, b.stride), dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            if pre == "copy":  # a device copy of the stats rows into an existing buffer
                C.check(L.st_copy(ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(b._views.stats),
                                  scratch.numel() * 4, b._stream()))
            elif pre == "torchsum":  # a torch reduction over an existing tensor
                int(scratch.sum())
            else:  # a new device allocation
                torch.empty(20 << 20, dtype=torch.uint8, device=dev)
        if pre != "none":
            torch.cuda.synchronize()
            if pre.startswith("sleep"):
                time.sleep(float(pre[5:]) * 1e-3)
        if pre != "plock_done":
            sp0 = spawned() if pre == "plock" else 0
        with torch.cuda.stream(s):
            e0.record(s)
            for c in range(K // CH):
                C.check(L.st_rollout(ctx, CH, ap[WU + c * CH], pp[0], None, pp[1], pp[2], sp))
            e1.record(s)
        torch.cuda.synchronize()
        res.append(f"rollout {e0.elapsed_time(e1) * 1e3 / (K // CH * CH):.3f}")
        if pre == "plock":
            res.append(f"(rollout p_lock {(spawned() - sp0) / (n * (K // CH) * CH):.4f})")
    del g
    b.close()
print(os.path.basename(os.environ.get("ST_LIB", "in-tree")), " ".join(res), "us/step", flush=True)
