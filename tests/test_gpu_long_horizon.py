"""The timed bench workload itself, at full size and over the bench's horizon,
bit-exact against the C oracle (VERDICT r1 "next" #1).

bench.py times 65,536 envs (seeds 1000 + e), synthetic actions
splitmix64(0x5EED ^ (t << 32 ^ e)) % 7, same-step auto-reset, W eager warm-up
st_step launches and then K st_step launches captured in one hipGraph.  These
tests run exactly that (W = 100, K = 4,000: a second MT generation switch for
most envs, boards at full occupancy, every auto-reset path) with each step's
outputs written to its own slot, and compare every step's reward, done and
packed obs, then the final board / piece / counters / MT19937 state, with the
oracle (TetrisEngine.step restated, tetris_env.py:243-304; CPython's random,
:183-191), for BASELINE configs C3 and C4.  The same for st_rollout: 10
launches of 100 steps.  The oracle runs on host threads over env slices
(ctypes releases the GIL), so the check takes seconds.
"""
import ctypes
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N, W, H = 65536, 10, 20
WU, K = 100, 4000
SEED_BASE, ASEED = 1000, 0x5EED
CONFIGS = {
    "c3": dict(),
    "c4": dict(advanced_clears=True, penalise_holes_increase=True, penalise_height_increase=True),
}


def _threads():
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(16, n))


class ParallelOracle:
    """N oracle envs split into contiguous slices, one host thread each;
    global env index e keeps seed SEED_BASE + e and the action stream of e."""

    def __init__(self, n, kw, parts=None):
        parts = parts or _threads()
        bounds = np.linspace(0, n, parts + 1).astype(int)
        self.sl = [(int(a), int(b)) for a, b in zip(bounds[:-1], bounds[1:]) if b > a]
        kw = dict(dict(width=W, height=H), **kw)  # (a board other than 10x20: width / height in kw)
        self.obs = [O.OracleBatch(b - a, [SEED_BASE + a + e for e in range(b - a)], **kw)
                    for a, b in self.sl]
        for ob in self.obs:
            ob.reset()
        self.pool = ThreadPoolExecutor(len(self.sl))

    def rollout(self, t0, T, obs=True, stats=False):
        def one(i):
            a, b = self.sl[i]
            acts = O.splitmix64_actions(ASEED, t0, T, b - a, offset=a)
            return self.obs[i].rollout(acts, want_obs=obs, want_stats=stats)
        rs = list(self.pool.map(one, range(len(self.sl))))
        keys = ("reward", "done") + (("obs",) if obs else ()) + (("stats",) if stats else ())
        return {k: np.concatenate([r[k] for r in rs], axis=1) for k in keys}

    def final_state(self):
        """Structured view of every env (Env struct fields) in global order."""
        return np.concatenate([np.ctypeslib.as_array(ob.envs) for ob in self.obs])

    def close(self):
        self.pool.shutdown()


def _pack_board(board_u8):
    """oracle board [n][OR_MAX_W][OR_MAX_H] u8 -> packed columns [W][n] u32 (bit y of word x)."""
    b = (board_u8[:, :W, :H] != 0).astype(np.uint64)
    return (b << np.arange(H, dtype=np.uint64)).sum(axis=2).astype(np.uint32).T


def _seeded_words(n):
    """random.seed(SEED_BASE + e) words of every env (the oracle's seeding)."""
    out = np.empty((n, 624), np.uint32)
    for e in range(n):
        out[e] = np.ctypeslib.as_array(O.MTRandom(SEED_BASE + e)._mt.mt)
    return out


def _twist_np(w):
    """One MT19937 refill of every row (CPython genrand_uint32 at index 624)."""
    w = w.astype(np.uint32).copy()
    for k in range(624):
        y = (w[:, k] & np.uint32(0x80000000)) | (w[:, (k + 1) % 624] & np.uint32(0x7FFFFFFF))
        w[:, k] = w[:, (k + 397) % 624] ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908B0DF),
                                                                       np.uint32(0))
    return w


def _check_final(eng, orc):
    st = eng.get_state()  # st_mt_sync first: CPython's exact MT state
    ref = orc.final_state()
    stats = st["stats"]
    for row, field in ((0, "time"), (1, "score"), (2, "lines_cleared"), (3, "holes"),
                       (4, "piece_height"), (5, "n_deaths")):
        assert np.array_equal(stats[row], ref[field]), field
    assert np.array_equal(stats[6:13].T, ref["counts"]), "shape counts"
    p = st["piece"]
    for name, got in (("shape_id", p & 7), ("rot", (p >> 3) & 3), ("ax", (p >> 5) & 63),
                      ("ay", (p >> 11) & 63), ("lock", p >> 17)):
        assert np.array_equal(got.astype(np.int64), ref[name].astype(np.int64)), name
    assert np.array_equal(st["board"], _pack_board(ref["board"])), "board"
    assert np.array_equal(stats[13], ref["rng"]["index"]), "MT index"
    assert np.array_equal(st["mt"], ref["rng"]["mt"].astype(np.uint32)), "MT words"


def _compare(t0, got_r, got_d, got_o, ref):
    assert np.array_equal(got_r, ref["reward"]), f"reward, steps {t0}.."
    assert np.array_equal(got_d.astype(np.uint8), ref["done"]), f"done, steps {t0}.."
    bad = np.argwhere((got_o.transpose(0, 2, 1) != ref["obs"]).any(axis=2))
    assert bad.size == 0, f"obs mismatch at (step, env) {bad[:4] + [t0, 0]}"


@pytest.mark.parametrize("config,launch", [("c3", "eager"), ("c3", "graph"), ("c4", "eager")])
def test_bench_workload_st_step(config, launch):
    """bench.py's headline region (eager: the default; graph: `--launch
    graph`, K launches captured in one hipGraph and replayed).  In the graph
    case the outputs of the timed steps hold a sentinel after the capture
    (capturing runs nothing) and the oracle's values after the replay: the
    compared steps really came from the graph."""
    import gym_simpletetris_amd as G
    from gym_simpletetris_amd import _lib as C
    dev = torch.device("cuda", 0)
    kw = CONFIGS[config]
    eng = G.TetrisBatch(N, autoreset="same_step", seeds=[SEED_BASE + e for e in range(N)],
                        device=dev, width=W, height=H, **kw)
    T = WU + K
    acts = torch.empty((T, N), dtype=torch.uint8, device=dev)
    for t in range(T):
        eng.gen_actions(t, ASEED, out=acts[t])
    eng.reset()
    SENT = -12345
    obs = torch.full((T, W, N), SENT, dtype=torch.int32, device=dev)
    rew = torch.full((T, N), SENT, dtype=torch.int32, device=dev)
    done = torch.full((T, N), 7, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    L, ctx = eng._L, eng._ctx
    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)

    def launch_step(t):
        C.check(L.st_step(ctx, ctypes.c_void_p(acts[t].data_ptr()), ctypes.c_void_p(obs[t].data_ptr()),
                          ctypes.c_void_p(rew[t].data_ptr()), ctypes.c_void_p(done[t].data_ptr()), sp))
    with torch.cuda.stream(s):
        for t in range(WU):  # bench warm-up: eager launches
            launch_step(t)
    torch.cuda.synchronize(dev)
    if launch == "graph":
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):  # bench --launch graph: one graph of K launches
            for t in range(WU, T):
                launch_step(t)
        torch.cuda.synchronize(dev)
        # captured, not run: every timed step's outputs still hold the sentinel
        assert bool((rew[WU:] == SENT).all()) and bool((obs[WU:] == SENT).all()) and bool((done[WU:] == 7).all())
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize(dev)
        del g
    else:
        assert launch == "eager"
        with torch.cuda.stream(s):  # bench default: K eager launches
            for t in range(WU, T):
                launch_step(t)
        torch.cuda.synchronize(dev)
    assert not bool((rew == SENT).any()) and not bool((done == 7).any())
    orc = ParallelOracle(N, kw)
    try:
        CH = 100
        for t0 in range(0, T, CH):
            ref = orc.rollout(t0, CH)
            _compare(t0, rew[t0:t0 + CH].cpu().numpy(), done[t0:t0 + CH].cpu().numpy(),
                     obs[t0:t0 + CH].cpu().numpy().view(np.uint32), ref)
        _check_final(eng, orc)
        # the regime the bench times: most envs went past their first generation
        fin = orc.final_state()["rng"]["mt"].astype(np.uint32)
        gen1 = _twist_np(_seeded_words(N))
        assert (fin != gen1).any(axis=1).mean() > 0.5
    finally:
        orc.close()
        eng.close()


def test_c2_shape_eager_long():
    """BASELINE C2 at its own shape: 4,096 10x20 boards, C3 (default)
    rewards, same-step auto-reset, 1,200 eager st_step launches (one per
    step, as bench.py times C2), every step's reward / done / packed obs and
    the final state bit-exact against the oracle."""
    import gym_simpletetris_amd as G
    from gym_simpletetris_amd import _lib as C
    n, T = 4096, 1200
    dev = torch.device("cuda", 0)
    eng = G.TetrisBatch(n, autoreset="same_step", seeds=[SEED_BASE + e for e in range(n)],
                        device=dev, width=W, height=H)
    acts = torch.empty((T, n), dtype=torch.uint8, device=dev)
    for t in range(T):
        eng.gen_actions(t, ASEED, out=acts[t])
    eng.reset()
    obs = torch.empty((T, W, n), dtype=torch.int32, device=dev)
    rew = torch.empty((T, n), dtype=torch.int32, device=dev)
    done = torch.empty((T, n), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    L, ctx = eng._L, eng._ctx
    sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for t in range(T):
        C.check(L.st_step(ctx, ctypes.c_void_p(acts[t].data_ptr()), ctypes.c_void_p(obs[t].data_ptr()),
                          ctypes.c_void_p(rew[t].data_ptr()), ctypes.c_void_p(done[t].data_ptr()), sp))
    torch.cuda.synchronize(dev)
    orc = ParallelOracle(n, {})
    try:
        CH = 200
        for t0 in range(0, T, CH):
            ref = orc.rollout(t0, CH)
            _compare(t0, rew[t0:t0 + CH].cpu().numpy(), done[t0:t0 + CH].cpu().numpy(),
                     obs[t0:t0 + CH].cpu().numpy().view(np.uint32), ref)
        _check_final(eng, orc)
        assert int(done.sum()) > n  # episodes turned over inside the compared span
    finally:
        orc.close()
        eng.close()


@pytest.mark.parametrize("config", sorted(CONFIGS))
def test_bench_workload_st_rollout(config):
    import gym_simpletetris_amd as G
    dev = torch.device("cuda", 0)
    kw = CONFIGS[config]
    eng = G.TetrisBatch(N, autoreset="same_step", seeds=[SEED_BASE + e for e in range(N)],
                        device=dev, width=W, height=H, **kw)
    CH, NL = 100, 10
    acts = torch.empty((CH * NL, N), dtype=torch.uint8, device=dev)
    for t in range(CH * NL):
        eng.gen_actions(t, ASEED, out=acts[t])
    eng.reset()
    orc = ParallelOracle(N, kw)
    buf = {}
    try:
        for c in range(NL):
            o, r, d = eng.rollout(acts[c * CH:(c + 1) * CH], obs="packed", out=buf)
            ref = orc.rollout(c * CH, CH)
            _compare(c * CH, r.cpu().numpy(), d.cpu().numpy(), o.cpu().numpy().view(np.uint32), ref)
        _check_final(eng, orc)
    finally:
        orc.close()
        eng.close()


@pytest.mark.parametrize("config", sorted(CONFIGS))
def test_rollout_large_batch_two_wave_kernel(config):
    """st_rollout above 4 workgroups per CU runs the two-wave rollout kernel
    (launch_rollout's choice; the three-wave kernel below it): 2x the CUs'
    4-workgroup batch plus a ragged tail, 3 launches x 100 steps, every step's
    outputs and the final state bit-exact against the oracle."""
    import gym_simpletetris_amd as G
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    n = 2 * 4 * 64 * cus + 37
    assert n > 4 * 64 * cus
    kw = CONFIGS[config]
    eng = G.TetrisBatch(n, autoreset="same_step", seeds=[SEED_BASE + e for e in range(n)],
                        device=dev, width=W, height=H, **kw)
    CH, NL = 100, 3
    acts = torch.empty((CH * NL, n), dtype=torch.uint8, device=dev)
    for t in range(CH * NL):
        eng.gen_actions(t, ASEED, out=acts[t])
    eng.reset()
    orc = ParallelOracle(n, kw)
    buf = {}
    try:
        for c in range(NL):
            o, r, d = eng.rollout(acts[c * CH:(c + 1) * CH], obs="packed", out=buf)
            ref = orc.rollout(c * CH, CH)
            _compare(c * CH, r.cpu().numpy(), d.cpu().numpy(), o.cpu().numpy().view(np.uint32), ref)
        _check_final(eng, orc)
    finally:
        orc.close()
        eng.close()


@pytest.mark.parametrize("n,steps", [(65537, 600), (1 << 20, 24)])
def test_ragged_and_large_batches(n, steps):
    """A ragged batch (65,537 envs: the last wave holds one real env, the
    stride is padded) over 600 graph-replayed steps, and 2^20 envs (16x the
    headline batch) over 24 steps, both bit-exact vs the oracle, C4 scoring."""
    import gym_simpletetris_amd as G
    from gym_simpletetris_amd import _lib as C
    dev = torch.device("cuda", 0)
    kw = CONFIGS["c4"]
    eng = G.TetrisBatch(n, autoreset="same_step", seeds=[SEED_BASE + e for e in range(n)],
                        device=dev, width=W, height=H, **kw)
    acts = torch.empty((steps, n), dtype=torch.uint8, device=dev)
    for t in range(steps):
        eng.gen_actions(t, ASEED, out=acts[t])
    eng.reset()
    obs = torch.empty((steps, W, n), dtype=torch.int32, device=dev)
    rew = torch.empty((steps, n), dtype=torch.int32, device=dev)
    done = torch.empty((steps, n), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    L, ctx = eng._L, eng._ctx
    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for t in range(steps):
            C.check(L.st_step(ctx, ctypes.c_void_p(acts[t].data_ptr()), ctypes.c_void_p(obs[t].data_ptr()),
                              ctypes.c_void_p(rew[t].data_ptr()), ctypes.c_void_p(done[t].data_ptr()), sp))
    with torch.cuda.stream(s):
        g.replay()
    torch.cuda.synchronize(dev)
    del g
    orc = ParallelOracle(n, kw)
    try:
        CH = 100
        for t0 in range(0, steps, CH):
            T = min(CH, steps - t0)
            ref = orc.rollout(t0, T)
            _compare(t0, rew[t0:t0 + T].cpu().numpy(), done[t0:t0 + T].cpu().numpy(),
                     obs[t0:t0 + T].cpu().numpy().view(np.uint32), ref)
        _check_final(eng, orc)
    finally:
        orc.close()
        eng.close()


def test_soak_many_generations():
    """100,000 steps of 8,192 envs (st_rollout, 1,000 steps per launch): ~40
    MT generation switches and ~1,800 episodes per env; every step's
    reward and done, then the final board / piece / counters / MT state,
    bit-exact against the oracle (C4 scoring)."""
    import gym_simpletetris_amd as G
    n, T, CH = 8192, 100000, 1000
    kw = CONFIGS["c4"]
    eng = G.TetrisBatch(n, autoreset="same_step", seeds=[SEED_BASE + e for e in range(n)],
                        width=W, height=H, **kw)
    eng.reset()
    orc = ParallelOracle(n, kw)
    acts = torch.empty((CH, n), dtype=torch.uint8, device=eng.device)
    try:
        deaths = 0
        for t0 in range(0, T, CH):
            for t in range(CH):
                eng.gen_actions(t0 + t, ASEED, out=acts[t])
            _, r, d = eng.rollout(acts, obs="none")
            ref = orc.rollout(t0, CH, obs=False)
            assert np.array_equal(r.cpu().numpy(), ref["reward"]), f"reward, steps {t0}.."
            dn = d.cpu().numpy().astype(np.uint8)
            assert np.array_equal(dn, ref["done"]), f"done, steps {t0}.."
            deaths += int(dn.sum())
        _check_final(eng, orc)
        assert deaths > 1000 * n  # the episodes really turned over
        fin = orc.final_state()["rng"]["mt"].astype(np.uint32)
        gen = _twist_np(_seeded_words(n))
        for _ in range(12):  # far past them: none of the first twelve generations remains
            assert not (fin == gen).all(axis=1).any()
            gen = _twist_np(gen)
    finally:
        orc.close()
        eng.close()
