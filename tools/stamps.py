"""Phase split of the step kernel from in-kernel s_memtime stamps (diagnostic
build: ST_STAMPS=1).  Prints median cycles per phase over waves and steps."""
import ctypes
import os
import sys

os.environ["ST_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gym_simpletetris_amd as G  # noqa: E402

f32 = "--f32" in sys.argv
n = 65536
b = G.TetrisBatch(n, autoreset="same_step", seeds=[1000 + e for e in range(n)])
b.reset()
nw = b.stride // 64
buf = np.zeros(nw * 8, np.uint64)
names = ["loads", "action+drop", "lock path", "draw", "obs+stores issue", "f32 block", "store drain"]
acc = []
for t in range(300):
    b.step(b.gen_actions(t, 0x5EED), obs="f32" if f32 else "packed")
    if t >= 100:
        b._L.st_debug_stamps(b._ctx, ctypes.c_void_p(buf.ctypes.data), buf.size)
        st = buf.reshape(nw, 8).astype(np.int64)
        acc.append(np.diff(st, axis=1))
a = np.concatenate(acc)
tot = (a.sum(1))
print(f"f32={f32} waves={nw} steps=200  total cycles median {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max()}")
for i, nm in enumerate(names):
    print(f"  {nm:18s} median {np.median(a[:, i]):7.0f}  mean {a[:, i].mean():7.0f}  p90 {np.percentile(a[:, i], 90):7.0f}")
