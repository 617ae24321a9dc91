"""Fast A/B timing of one libsimpletetris.so build (ST_LIB=path): graph-replayed
st_step at 65,536 envs for C3 and C4 (the bench workload) and the packed
rollout, event time per step.  usage: ST_LIB=lib.so python tools/ab_step.py [K]"""
import ctypes
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
    b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev, **kw)
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
        with torch.cuda.stream(s):
            C.check(L.st_rollout(ctx, CH, ap[WU], pp[0], None, pp[1], pp[2], sp))
            e0.record(s)
            for c in range(K // CH):
                C.check(L.st_rollout(ctx, CH, ap[WU + c * CH], pp[0], None, pp[1], pp[2], sp))
            e1.record(s)
        torch.cuda.synchronize()
        res.append(f"rollout {e0.elapsed_time(e1) * 1e3 / (K // CH * CH):.3f}")
    del g
    b.close()
print(os.path.basename(os.environ.get("ST_LIB", "in-tree")), " ".join(res), "us/step", flush=True)
