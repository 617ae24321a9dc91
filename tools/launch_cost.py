"""Host time per ctypes st_step call (the bench's eager loop), beside a
trivial ctypes call into the same library, at 64 envs (the GPU never
limits) and 65,536 envs.  usage: [ST_LIB=...] python tools/launch_cost.py"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-simpletetris_amd")]
import gym_simpletetris_amd as G  # noqa: E402
G.tune_runtime()
import torch  # noqa: E402
from gym_simpletetris_amd import _lib as C  # noqa: E402

out = {"lib": os.path.basename(os.environ.get("ST_LIB", "libsimpletetris.so"))}
L = C.load()
N = 10000
t0 = time.perf_counter()
for _ in range(N):
    L.st_abi_version()
out["ctypes_trivial_us"] = (time.perf_counter() - t0) / N * 1e6
for n in (64, 65536):
    b = G.TetrisBatch(n, autoreset="same_step", seeds=range(n))
    b.reset()
    a = b.gen_actions(0, 1).clone()
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    ptrs = [ctypes.c_void_p(x.data_ptr()) for x in (a, b.obs, b.reward, b.done)]
    ctx = b._ctx
    fn = L.st_step
    for _ in range(50):
        fn(ctx, *ptrs, sp)
    torch.cuda.synchronize()
    K = 2000
    t0 = time.perf_counter()
    for _ in range(K):
        fn(ctx, *ptrs, sp)
    t1 = time.perf_counter()
    s.synchronize()
    t2 = time.perf_counter()
    out[f"st_step_host_us_n{n}"] = (t1 - t0) / K * 1e6
    out[f"st_step_wall_us_n{n}"] = (t2 - t0) / K * 1e6
    b.close()
print(json.dumps(out))
