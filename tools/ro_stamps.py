"""Phase split of the st_rollout kernel from in-kernel s_memtime stamps
(diagnostic instantiation: ST_STAMPS=1 at st_create; the stamp build adds
~10% to the waves' cycles).  Each wave sums, per phase, the cycles between
consecutive stamps over the launch's steps; this prints the mean cycles per
step of every phase for the logic and the draw wave (median over workgroups),
65,536 envs, C3 rewards, 100-step launches, uniform splitmix64 actions.

usage: python tools/ro_stamps.py [CH] [launches]"""
import ctypes
import os
import sys

os.environ["ST_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402

CH = int(sys.argv[1]) if len(sys.argv) > 1 else 100
NL = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n = 65536
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)])
b.reset()
nw = b.stride // 64
W = 48  # kStampWords
buf = np.zeros(nw * W, np.uint64)
acts = torch.stack([b.gen_actions(t, 0x5EED).clone() for t in range(CH * NL)])
out = {}
# phases in execution order, by the stamp index that ends them
LOGIC = [(1, "step start (action load)"), (2, "action + drop"), (3, "queue / planes wait"),
         (4, "lock path"), (5, "reward/done + mask"), (6, "obs planes + state")]
DRAW = [(1, "round start"), (2, "chunk issue + mask wait"), (5, "draw"), (3, "ring + publish"),
        (6, "chunk bookkeeping"), (7, "window reload wait"), (4, "merge + reload issue")]
OUT = [(1, "wait for the planes"), (3, "planes read + obs stores"), (4, "reward/done/ep stores"),
       (5, "chunk: wait + twist + store"), (2, "next chunk issue")]
res = []
for c in range(NL):
    b.rollout(acts[c * CH:(c + 1) * CH], obs="packed", out=out)
    torch.cuda.synchronize()
    if c == 0:
        continue  # warm-up launch
    b._L.st_debug_stamps(b._ctx, ctypes.c_void_p(buf.ctypes.data), buf.size)
    res.append(buf.reshape(nw, W).astype(np.int64).copy())
r = np.stack(res)  # [launch, wg, 32]
steps = r[0, 0, 13]
print(f"st_rollout stamps: {n} envs, {steps} steps per launch, {len(res)} launches; "
      f"mean cycles per step (median over workgroups)")
for name, base, phases in (("logic wave", 0, LOGIC), ("draw wave", 16, DRAW), ("output wave", 32, OUT)):
    tot = 0.0
    print(f"{name}:")
    for i, nm in phases:
        v = np.median(r[:, :, base + i]) / steps
        tot += v
        print(f"  {nm:26s} {v:8.0f}")
    span = np.median(r[:, :, base + 12]) * 10.0 / steps  # s_memrealtime: 100 MHz -> ns
    print(f"  {'sum':26s} {tot:8.0f}   (wave life {span:.0f} ns per step)")
