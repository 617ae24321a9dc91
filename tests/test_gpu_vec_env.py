"""TetrisVecEnv's autoreset conventions and info snapshot (st_step_vec)
against the C oracle, at BASELINE's full 65,536 envs (VERDICT r3 "next" #2,
#4).

gym's vector-env convention (the default autoreset_obs='reset'):
an env that died in a step is reset inside it; the step returns its RESET
observation -- the empty board clear() returns (tetris_env.py:306-315,
:405-411) -- and its terminal observation (what the reference's step returned,
:301-302) is in info['final_observation'], valid where
info['_final_observation'].  autoreset_obs='terminal' returns the terminal obs
itself.  The info counters come from the snapshot the step kernel writes
(get_info, :232-241); ep_* hold the finished episode's counters where done.
The oracle's per-step stats are the counters before its auto-reset, so for a
done env the info must show clear()'s zeros (deaths kept) and the ep_* rows
the oracle's terminal counters.
"""
import numpy as np
import pytest
import torch

from test_gpu_long_horizon import ASEED, SEED_BASE, ParallelOracle
from test_gpu_parity import _engine

pytestmark = pytest.mark.gpu

W, H = 10, 20


C4 = dict(advanced_clears=True, penalise_holes_increase=True, penalise_height_increase=True)


def _unpack_f32(words, h=H):
    """packed obs [n][W] u32 -> float32 [n][W][h]."""
    return ((words[:, :, None] >> np.arange(h, dtype=np.uint32)) & 1).astype(np.float32)


def _check_info(info, ref_st, done, t):
    st = ref_st  # [n][8]: time, score, lines, holes, deaths, piece id, height, lock (before the reset)
    zero = np.zeros_like(st[:, 0])
    want = {"time": np.where(done, zero, st[:, 0]), "score": np.where(done, zero, st[:, 1]),
            "lines_cleared": np.where(done, zero, st[:, 2]), "holes": np.where(done, zero, st[:, 3]),
            "deaths": st[:, 4], "piece_height": np.where(done, zero, st[:, 6]),
            "ep_time": np.where(done, st[:, 0], zero), "ep_score": np.where(done, st[:, 1], zero),
            "ep_lines": np.where(done, st[:, 2], zero), "ep_holes": np.where(done, st[:, 3], zero)}
    for k, v in want.items():
        assert np.array_equal(info[k].cpu().numpy(), v), (k, t)
    cp = info["current_piece"].cpu().numpy()
    assert np.array_equal(cp[~done], st[~done, 5]), ("current_piece", t)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,w,h,kw", [(65536, 10, 20, {}), (1001, 10, 20, {}), (1001, 9, 15, C4)])
def test_vec_env_conventions_vs_oracle(n, w, h, kw):
    """Both conventions side by side, packed obs, every step checked: reward,
    done, returned obs, final_observation and the info counters; at the end
    the shape counts and current piece of every env.  n = 1,001 runs the
    ragged store path (n % 4 != 0); 9x15 with the C4 scoring flags the
    runtime-size vector kernel (k_step<0, 0, ..., VEC>)."""
    G = _engine()
    T = 300 if n == 65536 else 400
    a = G.TetrisVecEnv(n, width=w, height=h, seed=SEED_BASE, obs_format="packed", **kw)  # autoreset_obs='reset'
    b = G.TetrisVecEnv(n, width=w, height=h, seed=SEED_BASE, obs_format="packed", autoreset_obs="terminal", **kw)
    a.reset()
    b.reset()
    orc = ParallelOracle(n, dict(kw, width=w, height=h))
    acts = torch.empty(n, dtype=torch.uint8, device=a.device)
    CH = 50
    ndone = 0
    try:
        for t0 in range(0, T, CH):
            ref = orc.rollout(t0, CH, stats=True)
            for i in range(CH):
                t = t0 + i
                a.engine.gen_actions(t, ASEED, out=acts)
                oa, ra, da, ia = a.step(acts)
                ob, rb, db, ib = b.step(acts)
                done = ref["done"][i].astype(bool)
                robs = ref["obs"][i]  # [n][W] terminal obs where done
                for r_, d_ in ((ra, da), (rb, db)):
                    assert np.array_equal(r_.cpu().numpy(), ref["reward"][i]), ("reward", t)
                    assert np.array_equal(d_.cpu().numpy(), done), ("done", t)
                got_a = oa.cpu().numpy().view(np.uint32).T
                want_a = np.where(done[:, None], 0, robs)
                assert np.array_equal(got_a, want_a), ("reset-convention obs", t)
                assert np.array_equal(ob.cpu().numpy().view(np.uint32).T, robs), ("terminal obs", t)
                assert np.array_equal(ia["_final_observation"].cpu().numpy(), done), t
                fin = ia["final_observation"].cpu().numpy().view(np.uint32).T
                assert np.array_equal(fin, np.where(done[:, None], robs, 0)), ("final_observation", t)
                assert "final_observation" not in ib
                _check_info(ia, ref["stats"][i], done, t)
                if i % 10 == 0:
                    _check_info(ib, ref["stats"][i], done, t)
                ndone += int(done.sum())
        fin_state = orc.final_state()
        for info in (ia, ib):
            assert np.array_equal(info["statistics"].cpu().numpy().T, fin_state["counts"]), "statistics"
            assert np.array_equal(info["current_piece"].cpu().numpy(), fin_state["shape_id"]), "current_piece"
    finally:
        orc.close()
        a.close()
        b.close()
    assert ndone > n // 10  # resets inside the compared span


@pytest.mark.timeout(200)
@pytest.mark.parametrize("obs_type,n,w,h,kw", [("ram", 4096, 10, 20, {}), ("grayscale", 4096, 10, 20, {}),
                                               ("ram", 1001, 9, 15, C4)])
def test_vec_env_f32_and_image_conventions(obs_type, n, w, h, kw):
    """float32 ram obs (fused in the step kernel) and grayscale obs under the
    reset convention: the returned obs of a done env is the reset obs (zeros /
    the empty board's image) and final_observation is the terminal obs in the
    same format; the rest equals the packed path's conversion.  9x15, n =
    1,001, C4 flags: the runtime-size kernel's generic float32 writer with
    the reset mask (its KM-masked word path)."""
    G = _engine()
    T = 200
    a = G.TetrisVecEnv(n, width=w, height=h, seed=SEED_BASE, obs_type=obs_type, **kw)
    p = G.TetrisVecEnv(n, width=w, height=h, seed=SEED_BASE, obs_format="packed", autoreset_obs="terminal", **kw)
    a.reset()
    p.reset()
    acts = torch.empty(n, dtype=torch.uint8, device=a.device)
    empty = torch.zeros((w, n), dtype=torch.int32, device=a.device)
    saw = 0
    for t in range(T):
        a.engine.gen_actions(t, ASEED, out=acts)
        oa, ra, da, ia = a.step(acts)
        op, rp, dp, _ = p.step(acts)
        assert torch.equal(ra, rp) and torch.equal(da, dp), t
        terminal = op.clone()
        ret = torch.where(dp.unsqueeze(0), empty, op)
        fin = torch.where(dp.unsqueeze(0), op, empty)
        if obs_type == "ram":
            want = torch.from_numpy(_unpack_f32(ret.cpu().numpy().view(np.uint32).T, h)).to(a.device)
            wfin = torch.from_numpy(_unpack_f32(fin.cpu().numpy().view(np.uint32).T, h)).to(a.device)
        else:
            want = p.engine.grayscale(ret, 84, 1).squeeze(-1)
            wfin = p.engine.grayscale(fin, 84, 1).squeeze(-1)
        assert torch.equal(oa, want), t
        if bool(dp.any()) or t % 25 == 0:
            assert torch.equal(ia["final_observation"], wfin), t
            saw += int(dp.sum())
        del terminal
    assert saw > 0
    a.close()
    p.close()


def test_vec_env_info_kept_across_steps():
    """copy=False (the fast path): an info held past later steps still
    reports its own step (VERDICT r3 "next" #4): the env reuses an output
    slot two steps later and gives the info object a copy first; one not
    held costs nothing."""
    G = _engine()
    n = 2048
    v = G.TetrisVecEnv(n, seed=7, obs_format="packed", copy=False)
    v.reset()
    for t in range(30):
        v.step(v.engine.gen_actions(t, 5))
    kept = v.step(v.engine.gen_actions(30, 5))[3]
    live = {k: x.clone() for k, x in v.engine.info_tensors().items()}  # the state right after step 30
    done30 = kept["_final_observation"].clone()
    fin30 = kept["final_observation"].clone()
    infos, lives = [], []
    for t in range(31, 40):
        infos.append(v.step(v.engine.gen_actions(t, 5))[3])
        lives.append(v.engine.info_tensors()["time"].clone())
    for k in ("time", "score", "lines_cleared", "holes", "deaths", "statistics"):
        assert torch.equal(kept[k], live[k]), k
    assert torch.equal(kept["_final_observation"], done30)
    assert torch.equal(kept["final_observation"], fin30)
    # every info of the loop still reports its own step (each was detached in turn)
    for i, (inf, tm) in enumerate(zip(infos, lives)):
        assert torch.equal(inf["time"], tm), i
    v.close()


@pytest.mark.parametrize("obs_format", ["packed", "f32"])
def test_vec_env_outputs_kept_across_steps(obs_format):
    """copy=True (the default, gym's SyncVectorEnv convention; the reference
    returns a fresh np.copy each step, tetris_env.py:302): step t's obs /
    reward / done / info held across three later steps are unchanged, and
    equal a copy=False twin's outputs cloned at step t."""
    G = _engine()
    n = 4096
    v = G.TetrisVecEnv(n, seed=11, obs_format=obs_format)
    u = G.TetrisVecEnv(n, seed=11, obs_format=obs_format, copy=False)
    assert v.copy and not u.copy
    v.reset()
    u.reset()
    held = []
    for t in range(40):
        acts = v.engine.gen_actions(t, 5).clone()
        ov, rv, dv, iv = v.step(acts)
        ou, ru, du, iu = u.step(acts)
        snap = (ou.clone(), ru.clone(), du.clone(), iu["time"].clone(), iu["final_observation"].clone())
        held.append(((ov, rv, dv, iv), snap))
        if len(held) > 4:
            (o, r, d, i), (so, sr, sd, stime, sfin) = held.pop(0)  # step t - 4's, after four later steps
            assert torch.equal(o, so) and torch.equal(r, sr) and torch.equal(d, sd), t
            assert torch.equal(i["time"], stime) and torch.equal(i["final_observation"], sfin), t
    v.close()
    u.close()


@pytest.mark.parametrize("obs_format", ["packed", "f32"])
def test_vec_env_copy_reuses_only_dropped_slots(obs_format):
    """copy=True reuses a recent step's output slot once nothing of it is
    referenced (an RL loop that drops each step's outputs allocates nothing
    per step), and never one the caller still holds in any form: a derived
    view of the obs, the reward tensor, an info tensor, the info itself.
    Every step's outputs equal a copy=False twin's, and the held pieces are
    unchanged ten steps later."""
    G = _engine()
    n = 2048
    v = G.TetrisVecEnv(n, seed=13, obs_format=obs_format)
    u = G.TetrisVecEnv(n, seed=13, obs_format=obs_format, copy=False)
    v.reset()
    u.reset()
    held = {}
    for t in range(60):
        acts = v.engine.gen_actions(t, 9).clone()
        ov, rv, dv, iv = v.step(acts)
        ou, ru, du, iu = u.step(acts)
        assert torch.equal(ov, ou) and torch.equal(rv, ru) and torch.equal(dv, du), t
        assert torch.equal(iv["score"], iu["score"]) and torch.equal(iv["final_observation"], iu["final_observation"]), t
        k = t % 5
        if t in (10, 20, 30, 40):  # keep one piece of this step's outputs, drop the rest
            piece = {10: ov[..., :7], 20: rv, 30: iv["lines_cleared"], 40: iv}[t]
            want = {10: ou[..., :7], 20: ru, 30: iu["lines_cleared"], 40: iu["time"]}[t].clone()
            held[t] = (piece, want)
        del ov, rv, dv, iv
        for t0, (piece, want) in held.items():
            got = piece["time"] if t0 == 40 else piece
            assert torch.equal(got, want), (t0, t)
        del k
    # the drop-everything steps ran on recycled slots
    assert v.slots_reused >= 60 - 4 - 8, v.slots_reused
    v.close()
    u.close()


def test_vec_env_reset_return_info_vs_oracle():
    """reset(return_info=True) (tetris_env.py:405-411): (obs, info) with the
    post-clear() counters -- time / score / lines / holes / piece_height 0,
    the new current_piece, deaths and statistics kept (:306-315) -- equal
    the oracle's after the same steps and a reset of every env."""
    G = _engine()
    n, T = 2048, 150
    v = G.TetrisVecEnv(n, seed=SEED_BASE, obs_format="packed", **C4)
    obs0, info0 = v.reset(return_info=True)
    assert int(info0["time"].abs().sum()) == 0 and int(obs0.abs().sum()) == 0
    orc = ParallelOracle(n, C4)
    try:
        orc.rollout(0, T, obs=False)
        acts = torch.empty(n, dtype=torch.uint8, device=v.device)
        for t in range(T):
            v.engine.gen_actions(t, ASEED, out=acts)
            v.step(acts)
        obs, info = v.reset(return_info=True)
        for ob in orc.obs:
            ob.reset()
        ref = orc.final_state()
    finally:
        orc.close()
    assert int(obs.abs().sum()) == 0
    for k, f in (("time", "time"), ("score", "score"), ("lines_cleared", "lines_cleared"), ("holes", "holes"),
                 ("piece_height", "piece_height"), ("deaths", "n_deaths"), ("current_piece", "shape_id")):
        assert np.array_equal(info[k].cpu().numpy(), ref[f]), k
    assert np.array_equal(info["statistics"].cpu().numpy().T, ref["counts"])
    assert int(info["deaths"].sum()) > 0 and int(info["ep_score"].abs().sum()) == 0
    v.close()
