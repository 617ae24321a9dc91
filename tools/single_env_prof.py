import os, sys, time, random, ctypes
sys.path.insert(0, os.path.join(os.getcwd(), "gym-simpletetris_amd"))
import torch, numpy as np
from gym_simpletetris_amd.envs.tetris_env import TetrisEnv
from gym_simpletetris_amd import _lib as C
env = TetrisEnv(obs_type="ram", rng="private", seed=0)
env.reset()
for i in range(300):
    if env.step(i % 7)[2]: env.reset()
eng = env.engine; L, ctx = eng._L, eng._ctx
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
po, pr, pd = (ctypes.c_void_p(t.data_ptr()) for t in (eng.obs, eng.reward, eng.done))
N = 2000
def t(label, fn):
    t0 = time.perf_counter()
    for _ in range(N): fn()
    print(f"{label:40s} {(time.perf_counter()-t0)/N*1e6:7.2f} us", flush=True)
t("st_step launch only", lambda: L.st_step(ctx, env._p_acts[3], po, pr, pd, s))
torch.cuda.synchronize()
t("torch stream synchronize (idle)", lambda: torch.cuda.current_stream().synchronize())
hip = ctypes.CDLL("libamdhip64.so")
t("hipStreamSynchronize (idle)", lambda: hip.hipStreamSynchronize(s))
def step_sync():
    L.st_step(ctx, env._p_acts[3], po, pr, pd, s); hip.hipStreamSynchronize(s)
t("st_step + hipStreamSynchronize", step_sync)
def step_export_sync():
    L.st_step(ctx, env._p_acts[3], po, pr, pd, s); L.st_export_env(ctx, 0, po, pr, pd, env._parts, env._rec_dst, s); hip.hipStreamSynchronize(s)
t("st_step + export + hipSync", step_export_sync)
def full():
    if env.step(3)[2]: env.reset()
t("TetrisEnv.step (ram, private)", full)
t("random.getstate()", random.getstate)
st = random.getstate()
t("getstate == cached", lambda: random.getstate() == st)
