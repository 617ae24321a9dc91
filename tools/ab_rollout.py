"""Fast timing of st_rollout for one libsimpletetris.so build (ST_LIB=path,
ST_ABLATE for the ablation build): 65,536 envs, C3 (default) rewards,
same-step auto-reset, L launches of CH steps each after one warm-up launch,
HIP-event time per step, packed (and optionally float32) obs.

usage: ST_LIB=lib.so [ST_ABLATE=n] python tools/ab_rollout.py [CH] [L] [f32]
prints one line: `<label> packed <us/step> [f32 <us/step>]`."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

CH = int(sys.argv[1]) if len(sys.argv) > 1 else 100
NL = int(sys.argv[2]) if len(sys.argv) > 2 else 20
F32 = len(sys.argv) > 3 and sys.argv[3] == "f32"
n = int(os.environ.get("AB_N", "65536"))
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)], device=dev)
acts = torch.empty(((NL + 1) * CH, n), dtype=torch.uint8, device=dev)
for t in range((NL + 1) * CH):
    b.gen_actions(t, 0x5EED, out=acts[t])
b.reset()
torch.cuda.synchronize()
L, ctx = b._L, b._ctx
o = torch.empty((CH, 10, n), dtype=torch.int32, device=dev)
r = torch.empty((CH, n), dtype=torch.int32, device=dev)
d = torch.empty((CH, n), dtype=torch.uint8, device=dev)
pp = [ctypes.c_void_p(x.data_ptr()) for x in (o, r, d)]
out = [os.environ.get("AB_LABEL", os.path.basename(os.environ.get("ST_LIB", "default")) +
                      ":ablate=" + os.environ.get("ST_ABLATE", "0"))]
for use_f32 in ((False, True) if F32 else (False,)):
    f = torch.empty((CH, n, 10, 20), dtype=torch.float32, device=dev) if use_f32 else None
    pf = ctypes.c_void_p(f.data_ptr()) if use_f32 else None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        C.check(L.st_rollout(ctx, CH, ctypes.c_void_p(acts[0].data_ptr()), pp[0], pf, pp[1], pp[2], sp))
        e0.record(s)
        for c in range(1, NL + 1):
            C.check(L.st_rollout(ctx, CH, ctypes.c_void_p(acts[c * CH].data_ptr()), pp[0], pf, pp[1], pp[2], sp))
        e1.record(s)
    torch.cuda.synchronize()
    out.append("%s %.3f" % ("f32" if use_f32 else "packed", e0.elapsed_time(e1) * 1e3 / (NL * CH)))
    del f
print(" ".join(out), flush=True)
