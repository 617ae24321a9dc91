import sys, os
sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'gym-simpletetris_amd')
import numpy as np, torch
import gym_simpletetris_amd as G
from oracle import oracle as O
src = open('tests/test_gpu_parity.py').read()
i = src.index('def _untemper'); j = src.index('@pytest.mark.parametrize("mode"')
ns = {}; exec(src[i:j], ns); _untemper = ns['_untemper']
for mode in ("step", "rollout"):
    n, T = 64, 40
    b = G.TetrisBatch(n, autoreset="same_step", seeds=range(n)); b.reset()
    ob = O.OracleBatch(n, list(range(n))); ob.reset()
    st = b.get_state(("mt", "stats")); mt, stats = st["mt"].copy(), st["stats"].copy()
    rej, acc = _untemper(0xFFFFFFFF), _untemper(0)
    cls = {}
    for i in range(n):
        idx = int(stats[13, i]); cls[i] = 3
        if i % 4 == 0 and idx + 21 <= 624:
            mt[i, idx:idx + 20] = rej; mt[i, idx + 20] = acc; cls[i] = 0
        elif i % 4 == 1:
            stats[13, i] = 621 + (i % 3); cls[i] = 1
        elif i % 4 == 2 and idx + 41 <= 624:
            mt[i, idx:idx + 18] = rej; mt[i, idx + 18] = acc; mt[i, idx + 19:idx + 40] = rej; mt[i, idx + 40] = acc; cls[i] = 2
        e = ob.envs[i]
        for k in range(624): e.rng.mt[k] = int(mt[i, k])
        e.rng.index = int(stats[13, i])
    b.set_state(mt=mt, stats=stats)
    chk = b.get_state(("mt", "stats"))
    print(mode, "upload ok:", np.array_equal(chk["mt"], mt), np.array_equal(chk["stats"], stats))
    acts = np.full((T, n), 2, np.uint8); acts[::3] = O.splitmix64_actions(5, 0, T, n)[::3]
    # oracle step by step recording mt index per step
    idx_ref = []
    ref_obs = []
    for t in range(T):
        r = ob.rollout(acts[t:t+1]); ref_obs.append(r["obs"][0]); idx_ref.append([ob.envs[i].rng.index for i in range(n)])
    if mode == "step":
        for t in range(T):
            obs, rew, done = b.step(torch.as_tensor(acts[t], device=b.device))
            o = obs.cpu().numpy().view(np.uint32).T
            s2 = b.get_state(("stats",))["stats"]
            bad = np.nonzero((o != ref_obs[t]).any(1))[0]
            if len(bad):
                for i in bad[:6]:
                    print("t", t, "env", i, "class", cls[i], "dev idx", s2[13, i], "ref idx", idx_ref[t][i], "counts dev", s2[6:13, i], "ref", list(ob.envs[i].counts))
                break
        else:
            print("step: all ok")
    else:
        obs, rew, done = b.rollout(torch.as_tensor(acts, device=b.device))
        o = obs.cpu().numpy().view(np.uint32).transpose(0, 2, 1)
        for t in range(T):
            bad = np.nonzero((o[t] != ref_obs[t]).any(1))[0]
            if len(bad):
                print("rollout first bad t", t, "envs", bad[:10], [cls[i] for i in bad[:10]]); break
        else:
            print("rollout: all ok")
