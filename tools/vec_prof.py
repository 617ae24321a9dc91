import os, sys, time, ctypes
sys.path.insert(0, os.path.join(os.getcwd(), "gym-simpletetris_amd"))
import torch
import gym_simpletetris_amd as G
from gym_simpletetris_amd.envs.tetris_env import VecInfo
n = 65536
v = G.TetrisVecEnv(n, seed=1, obs_format="packed", validate_actions=False)
v.reset()
a = torch.randint(0, 7, (n,), dtype=torch.uint8, device=v.device)
dev = v.device
N = 3000
def t(label, fn):
    for _ in range(100): fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N): fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{label:34s} host {(t1-t0)/N*1e6:7.2f} us  wall {(t2-t0)/N*1e6:7.2f} us", flush=True)
t("vec.step", lambda: v.step(a))
t("engine.step packed", lambda: v.engine.step(a, obs="packed"))
t("VecInfo()", lambda: VecInfo(v.engine))
t("engine._actions", lambda: v.engine._actions(a))
t("current_stream ptr", lambda: ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
def ctx():
    with torch.cuda.device(dev):
        pass
t("torch.cuda.device ctx", ctx)
L, c = v.engine._L, v.engine._ctx
po, pr, pd, pa = (ctypes.c_void_p(x.data_ptr()) for x in (v.engine.obs, v.engine.reward, v.engine.done, a))
sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
t("raw st_step", lambda: L.st_step(c, pa, po, pr, pd, sp))
