"""Round 5 diagnostic: st_rollout's per-launch time against the envs' MT
generation phase.  Every env is seeded at the same time and draws at about
the same rate, so the grid's next-generation building (the output wave's
chunks, one per two steps while a wave has an incomplete successor) comes and
goes in phase across the whole grid.  Pass 1 times NL launches of 100 steps
(an event behind each, nothing between them); pass 2 replays the same
deterministic sequence on a fresh engine and copies the MT word row after
each launch, giving per launch: the share of envs whose successor is
incomplete (pg < 624) and the mean CPython index."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

n, CH = 65536, 100
NL = int(os.environ.get("NL", "80"))
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
T = (NL + 1) * CH


def run(record_phase):
    eng = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
    L, ctx = eng._L, eng._ctx
    acts = torch.empty((T, n), dtype=torch.uint8, device=dev)
    for t in range(T):
        eng.gen_actions(t, 0x5EED, out=acts[t])
    eng.reset()
    torch.cuda.synchronize()
    o = torch.empty((CH, 10, n), dtype=torch.int32, device=dev)
    r = torch.empty((CH, n), dtype=torch.int32, device=dev)
    d = torch.empty((CH, n), dtype=torch.uint8, device=dev)
    pp = [ctypes.c_void_p(x.data_ptr()) for x in (o, r, d)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(NL + 1)]
    snap = torch.empty((NL, eng.stride), dtype=torch.int32, device=dev) if record_phase else None
    src = eng._views.stats + C.STAT["mt_index"] * eng.stride * 4
    with torch.cuda.stream(s):
        for e in ev:
            e.record(s)
        torch.cuda.synchronize()
        ev[0].record(s)
        for c in range(NL):
            C.check(L.st_rollout(ctx, CH, ctypes.c_void_p(acts[c * CH].data_ptr()), pp[0], None, pp[1], pp[2], sp))
            ev[c + 1].record(s)
            if record_phase:
                C.check(L.st_copy(ctypes.c_void_p(snap[c].data_ptr()), ctypes.c_void_p(src), eng.stride * 4, sp))
    torch.cuda.synchronize()
    us = [ev[c].elapsed_time(ev[c + 1]) * 1e3 / CH for c in range(NL)]
    out = None
    if record_phase:
        w = snap[:, :n].cpu().numpy().astype("uint32")
        pg = (w >> 10) & 0x3FF
        idx = w & 0x3FF
        out = ((pg < 624).mean(axis=1), idx.mean(axis=1))
    eng.close()
    return us, out


us, _ = run(False)
us2, (building, idx) = run(True)
print("launch  us/step(pass1)  us/step(pass2,copies)  building  mean_idx")
for c in range(NL):
    print("%4d  %6.3f  %6.3f  %5.3f  %6.1f" % (c, us[c], us2[c], building[c], idx[c]))
import numpy as np  # noqa: E402
u, b = np.array(us[1:]), building[1:]
print("corr(us, building) = %.3f; mean us/step %.3f; building>0.5: %.3f, <0.2: %.3f" % (
    np.corrcoef(u, b)[0, 1], u.mean(), u[b > 0.5].mean() if (b > 0.5).any() else float("nan"),
    u[b < 0.2].mean() if (b < 0.2).any() else float("nan")))
