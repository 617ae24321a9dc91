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
W = 48  # kStampWords: logic wave words 0-15, draw wave 16-31 (32-47: the rollout output wave)
buf = np.zeros(nw * W, np.uint64)
rts = []
# logic wave: stamps 0 1 2 3 8 4 5 6 7 (8 sits between 3 and 4)
names = ["loads+B0", "action+drop", "B1+lock path", "early stores", "spawn-id wait", "obs+counters", "state stores issue", "store drain"]
# draw wave: stamps 0 1 2 10 9 4 11 6 7
dnames = ["loads+B0", "until L's action", "B1", "MT words wait", "draws", "commit", "state stores issue", "store drain"]
acc, dacc = [], []


def record():
    global names
    b._L.st_debug_stamps(b._ctx, ctypes.c_void_p(buf.ctypes.data), buf.size)
    full = buf.reshape(nw, W).astype(np.int64)
    if (full[:, 9] != 0).all():  # round 6's early stores: logic stamp 9 after them, before the lock path
        names = ["loads+B0", "action+drop", "B1+early stores", "lock path", "late stores", "spawn-id wait",
                 "obs+counters", "state stores issue", "store drain"]
        acc.append(np.diff(full[:, [0, 1, 2, 9, 3, 8, 4, 5, 6, 7]], axis=1))
    elif (full[:, 14] != 0).all() and (full[:, 15] != 0).all():  # round 6's split of the early-store phase
        names = ["loads+B0", "action+drop", "B1+lock path", "reward/done issue", "paint+LDS reads",
                 "obs+board stores", "spawn-id wait", "obs+counters", "state stores issue", "store drain"]
        acc.append(np.diff(full[:, [0, 1, 2, 3, 14, 15, 8, 4, 5, 6, 7]], axis=1))
    else:
        acc.append(np.diff(full[:, [0, 1, 2, 3, 8, 4, 5, 6, 7]], axis=1))
    dacc.append(np.diff(full[:, [16 + i for i in (0, 1, 2, 10, 9, 4, 11, 6, 7)]], axis=1))
    r = full[:, 10:15].copy()
    r[:, 4] = full[:, 30]  # draw kind (written by the draw wave)
    rts.append(np.concatenate([r, full[:, 28:30]], axis=1))


if "--graph" in sys.argv:
    # back-to-back launches as in bench.py: a hipGraph of 10 st_step calls,
    # replayed; the stamps are those of each replay's last step
    C = G._lib
    s = torch.cuda.Stream()
    acts = [b.gen_actions(t, 0x5EED).clone() for t in range(100 + 10 * 200)]
    obs = torch.empty((b.width, n), dtype=torch.int32, device=b.device)
    rew = torch.empty(n, dtype=torch.int32, device=b.device)
    done = torch.empty(n, dtype=torch.uint8, device=b.device)
    for t in range(100):
        b.step(acts[t])
    torch.cuda.synchronize()
    vp = ctypes.c_void_p
    sp = vp(s.cuda_stream)
    for rep in range(200):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for t in range(100 + 10 * rep, 110 + 10 * rep):
                C.check(b._L.st_step(b._ctx, vp(acts[t].data_ptr()), vp(obs.data_ptr()),
                                     vp(rew.data_ptr()), vp(done.data_ptr()), sp))
        g.replay()
        torch.cuda.synchronize()
        record()
        del g
else:
    for t in range(300):
        b.step(b.gen_actions(t, 0x5EED), obs="f32" if f32 else "packed")
        if t >= 100:
            record()
a = np.concatenate(acc)
tot = (a.sum(1))
print(f"f32={f32} waves={nw} steps=200  total cycles median {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max()}")
for i, nm in enumerate(names):
    print(f"  {nm:18s} median {np.median(a[:, i]):7.0f}  mean {a[:, i].mean():7.0f}  p90 {np.percentile(a[:, i], 90):7.0f}")
da = np.concatenate(dacc)
print(f"draw wave: total cycles median {np.median(da.sum(1)):.0f} p90 {np.percentile(da.sum(1), 90):.0f}")
for i, nm in enumerate(dnames):
    print(f"  {nm:18s} median {np.median(da[:, i]):7.0f}  mean {da[:, i].mean():7.0f}  p90 {np.percentile(da[:, i], 90):7.0f}")

# wave placement in time (s_memrealtime, 100 MHz => 10 ns ticks)
r = np.stack(rts)  # [steps, waves, 4]
t0 = r[:, :, 0] - r[:, :, 0].min(axis=1, keepdims=True)
t1 = r[:, :, 1] - r[:, :, 0].min(axis=1, keepdims=True)
ns = 10.0
print(f"wave start offset ns: median {np.median(t0)*ns:.0f} p90 {np.percentile(t0, 90)*ns:.0f} max {t0.max(1).mean()*ns:.0f} (mean over steps)")
print(f"wave end   offset ns: median {np.median(t1)*ns:.0f} p90 {np.percentile(t1, 90)*ns:.0f} max {t1.max(1).mean()*ns:.0f}")
print(f"wave life ns: median {np.median(t1 - t0)*ns:.0f}")
d0 = r[:, :, 5] - r[:, :, 0].min(axis=1, keepdims=True)
d1 = r[:, :, 6] - r[:, :, 0].min(axis=1, keepdims=True)
print(f"draw wave: start median {np.median(d0)*ns:.0f} ns, end median {np.median(d1)*ns:.0f} p90 {np.percentile(d1, 90)*ns:.0f} "
      f"max {d1.max(1).mean()*ns:.0f}; ends after its logic wave in {np.mean(d1 > t1)*100:.0f}% of workgroups")
xcc = r[0, :, 3] & 0xF
hw = r[0, :, 2]
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
print("waves per xcc", np.bincount(xcc, minlength=8).tolist())
print("distinct (xcc,se,cu):", len(set(zip(xcc.tolist(), se.tolist(), cu.tolist()))), " simd hist", np.bincount(simd, minlength=4).tolist())
for k in range(8):
    m = xcc == k
    if m.any():
        print(f"  xcc {k}: start median {np.median(t0[:, m])*ns:.0f} end max {t1[:, m].max(1).mean()*ns:.0f}")

# the slowest wave of each step (the kernel ends with it): which phase is long?
life = a.reshape(len(acc), nw, -1)
tot_w = life.sum(2)
slow = np.argmax(tot_w, axis=1)
sl = life[np.arange(len(acc)), slow]
print("slowest wave per step, mean cycles by phase (vs the median wave):")
for i, nm in enumerate(names):
    print(f"  {nm:18s} slowest {sl[:, i].mean():8.0f}   median wave {np.median(life[:, :, i]):7.0f}")
print(f"  {'total':18s} slowest {tot_w.max(1).mean():8.0f}   median wave {np.median(tot_w):7.0f}")
k = 10
top = np.sort(tot_w, axis=1)[:, -k:]
print(f"the {k} slowest waves per step: mean total {top.mean():.0f} cycles")

kind = r[:, :, 4]  # 1: a lane twisted its MT state, 2: a draw ran past the 8 prefetched words
for kd, nm in ((0, "plain"), (1, "twist"), (2, "past 8 words"), (3, "both")):
    m = kind == kd
    if m.any():
        dl = da.reshape(len(dacc), nw, -1)
        print(f"draw kind {nm:13s}: {m.sum() / len(acc):6.1f} waves/step, draw-wave draws median "
              f"{np.median(dl[:, :, 4][m]):6.0f}, logic total median {np.median(tot_w[m]):6.0f} cycles")
print("kind of the slowest wave per step:", np.bincount(kind[np.arange(len(acc)), slow], minlength=4).tolist())
