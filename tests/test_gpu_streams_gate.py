"""Round 6 surfaces on the GPU:

* validate_actions=True through the action gate (st_gate_actions /
  st_gate_wait): the reference's immediate KeyError (tetris_env.py:245,
  before TetrisEngine.step changes anything) without draining the stream --
  a rejected step leaves every env exactly as it was, and the steps around
  it equal an unvalidated twin's;
* TetrisVecEnv copy=True slot reuse honours consumer streams
  (record_stream) and follows the caller's holding depth;
* TetrisEnv's info['statistics'] is the env's one live shape-count dict
  (tetris_env.py:181, :199, :240): a held info sees later spawns, and counts
  written into it weight the next draws (:183-191), as in the reference --
  checked against the C oracle with the same counts written.
"""
import numpy as np
import pytest
import torch

from test_gpu_parity import _engine

pytestmark = pytest.mark.gpu


def _delay(ms_target: float = 30.0):
    """Queue roughly ms_target of GPU work on the current stream."""
    if hasattr(torch.cuda, "_sleep"):
        torch.cuda._sleep(int(ms_target * 2.0e6))  # ~2e6 cycles per ms
        return
    x = torch.randn(4096, 4096, device="cuda")
    for _ in range(8):
        x = x @ x


def _state(b):
    st = b.get_state(("board", "stats", "mt"))
    return {k: v.copy() for k, v in st.items()}


@pytest.mark.parametrize("obs", ["packed", "f32"])
def test_gate_rejects_before_any_state_change(obs):
    """TetrisBatch(validate_actions=True).step with device actions: a batch
    holding one action outside 0..6 (uint8 9, int64 -1 / 263, float 2.5 /
    nan) raises KeyError and changes no env (board, counters, MT state
    identical); the good steps around it equal an unvalidated twin's."""
    G = _engine()
    n = 1000
    a = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=True)
    b = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=False)
    a.reset()
    b.reset()
    step = (lambda eng, x: eng.step(x, obs=obs))
    for t in range(40):
        acts = b.gen_actions(t, 3).clone()
        oa, ra, da = step(a, acts)
        ob, rb, db = step(b, acts)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        if t in (10, 25):
            before = _state(a)
            good = b.gen_actions(100 + t, 3)
            bads = [good.clone(), good.to(torch.int64), good.to(torch.int64), good.to(torch.float32),
                    good.to(torch.float32)]
            bads[0][617] = 9
            bads[1][0] = -1
            bads[2][n - 1] = 263
            bads[3][500] = 2.5
            bads[4][3] = float("nan")
            for x in bads:
                with pytest.raises(KeyError):
                    step(a, x)
            after = _state(a)
            for k in before:
                assert np.array_equal(before[k], after[k]), (k, t)
    # in-range non-uint8 device actions pass the gate
    oa, ra, da = step(a, torch.arange(n, device=a.device) % 7)
    ob, rb, db = step(b, torch.arange(n, device=b.device) % 7)
    assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db)
    a.close()
    b.close()


def test_gate_ends_at_wait_even_without_its_step():
    """C ABI: a gate whose step launch failed (st_step with a null action
    pointer: ST_EINVAL before anything is queued) ends at st_gate_wait -- the
    next, ungated st_step is an ordinary step, not skipped by the stale
    answer (TetrisBatch.step and TetrisVecEnv.step end a gate the same way,
    _gate_abort, when their step launch raises)."""
    import ctypes
    G = _engine()
    from gym_simpletetris_amd import _lib as C
    n = 256
    a = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=False)
    b = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=False)
    a.reset()
    b.reset()
    L, ctx, vp = a._L, a._ctx, ctypes.c_void_p
    s = vp(torch.cuda.current_stream().cuda_stream)
    bad = torch.full((n,), 9, dtype=torch.uint8, device=a.device)
    assert L.st_gate_actions(ctx, vp(bad.data_ptr()), s) == 0
    o, r, d = (torch.empty((10, n), dtype=torch.int32, device=a.device),
               torch.empty(n, dtype=torch.int32, device=a.device), torch.empty(n, dtype=torch.uint8, device=a.device))
    assert L.st_step(ctx, None, vp(o.data_ptr()), vp(r.data_ptr()), vp(d.data_ptr()), s) == C.ST_EINVAL
    assert L.st_gate_wait(ctx) == 1  # the check saw the 9
    good = b.gen_actions(0, 5).clone()
    assert L.st_step(ctx, vp(good.data_ptr()), vp(o.data_ptr()), vp(r.data_ptr()), vp(d.data_ptr()), s) == 0
    ob, rb, db = b.step(good)
    torch.cuda.synchronize()
    assert torch.equal(o, ob) and torch.equal(r, rb) and torch.equal(d.bool(), db.bool())
    sa, sb = _state(a), _state(b)
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    a.close()
    b.close()


@pytest.mark.parametrize("obs_format,copy", [("packed", True), ("f32", True), ("packed", False)])
def test_gate_vec_env_and_abi(obs_format, copy):
    """TetrisVecEnv(validate_actions=True): a rejected step changes nothing
    and the env continues in lockstep with an unvalidated twin (packed and
    float32 obs, the reset obs / final_observation convention, both copy
    modes); the C ABI's gate calls in order (st_gate_wait without
    st_gate_actions: ST_ESTATE)."""
    G = _engine()
    from gym_simpletetris_amd import _lib as C
    n = 2048
    v = G.TetrisVecEnv(n, seed=21, obs_format=obs_format, validate_actions=True, copy=copy)
    u = G.TetrisVecEnv(n, seed=21, obs_format=obs_format, validate_actions=False, copy=copy)
    v.reset()
    u.reset()
    for t in range(60):
        acts = u.engine.gen_actions(t, 7).clone()
        if t % 20 == 19:
            bad = acts.clone()
            bad[t * 13 % n] = 200
            with pytest.raises(KeyError):
                v.step(bad)
        ov, rv, dv, iv = v.step(acts)
        ou, ru, du, iu = u.step(acts)
        assert torch.equal(ov, ou) and torch.equal(rv, ru) and torch.equal(dv, du), t
        assert torch.equal(iv["time"], iu["time"]) and torch.equal(iv["score"], iu["score"]), t
        assert torch.equal(iv["final_observation"], iu["final_observation"]), t
    L = v.engine._L
    assert L.st_gate_wait(v.engine._ctx) == C.ST_ESTATE
    v.close()
    u.close()


def test_record_stream_orders_slot_reuse():
    """copy=True: a consumer on another stream registered with
    record_stream() reads step t's obs behind ~30 ms of queued work and drops
    it at once; the env's next steps (which reuse that slot) wait for it on
    the device, so the consumer still reads step t's obs."""
    G = _engine()
    n = 8192
    v = G.TetrisVecEnv(n, seed=3, obs_format="packed")
    side = torch.cuda.Stream()
    v.record_stream(side)
    v.reset()
    for t in range(6):  # the pool settles: every step reuses the slot it dropped
        v.step(v.engine.gen_actions(t, 1))
    r0 = v.slots_reused
    obs, rew, done, info = v.step(v.engine.gen_actions(6, 1))
    want = obs.clone()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        _delay()
        got = obs.clone()
        got_r = rew.clone()
    want_r = rew.clone()
    del obs, rew, done, info
    for t in range(7, 15):
        v.step(v.engine.gen_actions(t, 1))  # these reuse the consumer's slot
    torch.cuda.synchronize()
    assert v.slots_reused > r0
    assert torch.equal(got, want) and torch.equal(got_r, want_r)
    v.close()


def test_record_stream_orders_copy_false_alternation():
    """copy=False: the env writes a slot again two steps later; a consumer
    registered with record_stream() that is still reading it behind queued
    work on its own stream keeps reading the step it was given."""
    G = _engine()
    n = 8192
    v = G.TetrisVecEnv(n, seed=5, obs_format="packed", copy=False)
    side = torch.cuda.Stream()
    v.record_stream(side)
    v.reset()
    for t in range(4):
        v.step(v.engine.gen_actions(t, 2))
    obs, rew, done, _ = v.step(v.engine.gen_actions(4, 2))
    want = obs.clone()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        _delay()
        got = obs.clone()
    for t in range(5, 9):
        v.step(v.engine.gen_actions(t, 2))  # the slot of step 4 is written again at step 6
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    v.close()


@pytest.mark.parametrize("depth", [1, 8])
def test_pool_follows_holding_depth(depth):
    """copy=True with every step's outputs kept for `depth` steps: the pool
    grows to depth + 1 slots and then reuses one per step (no allocation),
    and every kept output still equals a copy=False twin's at its step."""
    G = _engine()
    n = 4096
    v = G.TetrisVecEnv(n, seed=17, obs_format="packed")
    u = G.TetrisVecEnv(n, seed=17, obs_format="packed", copy=False)
    v.reset()
    u.reset()
    held = []
    T = 60
    for t in range(T):
        acts = v.engine.gen_actions(t, 4).clone()
        ov, rv, dv, iv = v.step(acts)
        ou, ru, du, iu = u.step(acts)
        held.append((ov, rv, iv, ou.clone(), ru.clone(), iu["score"].clone()))
        if len(held) > depth:
            o, r, i, so, sr, ss = held.pop(0)
            assert torch.equal(o, so) and torch.equal(r, sr) and torch.equal(i["score"], ss), t
            del o, r, i
        del ov, rv, dv, iv
    assert v.slots_reused >= T - (depth + 2), (v.slots_reused, depth)
    assert len(v._pool) <= depth + 1
    v.close()
    u.close()


def test_tetris_env_statistics_is_live_and_writable():
    """TetrisEnv: info['statistics'] is one dict for the env's life -- an
    info kept from an early step shows the latest counts -- and counts
    written into it take effect at the next draw, like writing into the
    reference's shape_counts; the C oracle with the same counts written
    agrees on every later reward, done, obs and current piece."""
    G = _engine()
    from oracle import oracle as O
    seed = 12345
    env = G.TetrisEnv(rng="private", seed=seed)
    orc = O.OracleBatch(1, [seed])
    obs = env.reset()
    orc.reset(0)
    rng = np.random.default_rng(7)
    first = None
    wrote = 0
    for t in range(600):
        a = int(rng.integers(0, 7))
        if t in (50, 200, 400):  # write into the live dict
            d = info["statistics"]
            d["I"] += 30 if t == 50 else 0
            d["T"] = 0 if t == 200 else d["T"] + 7
            if t == 400:
                d["O"] = d["O"] + 100
            orc.set_state(0, counts=[d[k] for k in O.SHAPE_NAMES])
            wrote += 1
        obs, r, done, info = env.step(a)
        robs, rr, rdone, _ = orc.step_one(0, a)
        assert r == rr and done == rdone, t
        assert np.array_equal(obs, robs.astype(np.float32)), t
        e = orc.envs[0]
        assert info["current_piece"] == O.SHAPE_NAMES[e.shape_id], t
        assert list(info["statistics"].values()) == [int(e.counts[k]) for k in range(7)], t
        if first is None:
            first = info
        assert first["statistics"] is info["statistics"]  # the same live dict
        if done:
            env.reset()
            orc.reset(0)
    assert wrote == 3
    with pytest.raises(ValueError):
        info["statistics"]["T"] = "many"
        env.step(0)
    env.close()


def test_unwire_shards_checks_out_buffers():
    """unwire_shards(out=...) validates every caller buffer before the kernel
    writes through its pointer: shape, dtype, device, contiguity."""
    from gym_simpletetris_amd.engine import unwire_shards
    dev = torch.device("cuda", 0)
    W, H, ng, shards = 10, 20, 199, 2
    recv = torch.zeros((shards, 8, 100), dtype=torch.int32, device=dev)
    good = (torch.empty((W, ng), dtype=torch.int32, device=dev), torch.empty(ng, dtype=torch.int32, device=dev),
            torch.empty(ng, dtype=torch.bool, device=dev))
    o, r, d = unwire_shards(recv, W, H, ng, out=good)
    assert o.data_ptr() == good[0].data_ptr()
    unwire_shards(recv, W, H, ng, out=(good[0], good[1], good[2].view(torch.uint8)))
    bad = [(good[0][:, :ng - 1], good[1], good[2]),                      # short obs
           (good[0], good[1].to(torch.int64), good[2]),                   # wrong dtype
           (good[0], good[1], torch.empty(ng - 5, dtype=torch.bool, device=dev)),
           (good[0].cpu(), good[1], good[2]),                             # wrong device
           (torch.empty((ng, W), dtype=torch.int32, device=dev).t(), good[1], good[2]),  # not contiguous
           (good[0], good[1])]
    for out in bad:
        with pytest.raises(ValueError):
            unwire_shards(recv, W, H, ng, out=out)
