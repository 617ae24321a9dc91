"""HIP engine parity: the C-ABI library (libsimpletetris.so) on the GPU vs the
reference's own outputs (tests/golden/*.npz) and the C oracle.  Bit-exact for
every field (integer / bit work: no tolerance)."""
import ctypes
import random

import numpy as np
import pytest
import torch

from oracle import oracle as O
from replay import GOLDEN, load_set, replay_crafted, replay_rollout

pytestmark = pytest.mark.gpu

ROLL = load_set("rollouts.npz")
GREEDY = load_set("greedy.npz")
CRAFTED = load_set("crafted.npz")
RENDER = load_set("render.npz")


def _engine():
    import gym_simpletetris_amd as G
    return G


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


class HipAdapter:
    """TetrisBatch(autoreset='none') behind the replay interface."""

    def __init__(self, n, seeds, kw):
        G = _engine()
        self.b = G.TetrisBatch(n, autoreset="none", seeds=seeds, **kw)
        self.n = n

    def reset(self, mask):
        m = torch.as_tensor(np.asarray(mask, np.uint8), device=self.b.device)
        self.b.reset(None if bool(np.all(mask)) else m)

    def set_state(self, i, init):
        st = self.b.get_state(("board", "piece", "stats"))
        st["board"][:, i] = init["board"]
        st["piece"][i] = init["piece"]
        s = st["stats"]
        s[0, i], s[1, i], s[2, i], s[3, i] = init["time"], init["score"], init["lines"], init["holes"]
        s[4, i], s[5, i] = init["height"], init["deaths"]
        s[6:13, i] = init["counts"]
        self.b.set_state(**st)

    def step(self, actions):
        obs, rew, done = self.b.step(torch.as_tensor(np.asarray(actions, np.uint8),
                                                     device=self.b.device), obs="packed")
        st = self.b.get_state(("board", "piece", "stats"))
        s = st["stats"]
        return dict(reward=rew.cpu().numpy(), done=done.cpu().numpy().astype(np.uint8),
                    time=s[0], score=s[1], lines=s[2], holes=s[3], height=s[4], deaths=s[5],
                    counts=s[6:13].T, piece=st["piece"],
                    obs=obs.cpu().numpy().view(np.uint32).T, board=st["board"].T)


def test_library_is_the_hip_build():
    G = _engine()
    from gym_simpletetris_amd import _lib
    L = _lib.load()
    assert L.st_abi_version() == _lib.ABI_VERSION
    b = G.TetrisBatch(3, seeds=[1, 2, 3])
    b.reset()
    b.step(np.zeros(3, np.uint8))
    torch.cuda.synchronize()


def _twist(words):
    """One MT19937 generation refill (CPython genrand_uint32 at index 624)."""
    w = [int(x) for x in words]
    for k in range(624):
        y = (w[k] & 0x80000000) | (w[(k + 1) % 624] & 0x7FFFFFFF)
        w[k] = w[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
    return np.array(w, dtype=np.uint32)


def test_device_mt19937_matches_cpython():
    """Seed kernel (init_by_array) == random.Random(seed).getstate() exactly
    (words and index 624), and its first generation == CPython's first 624
    outputs."""
    G = _engine()
    d = np.load(f"{GOLDEN}/mt19937.npz")
    seeds = [int(s) for s in d["seeds"]]
    b = G.TetrisBatch(len(seeds), seeds=seeds, autoreset="same_step")
    st = b.get_state(("mt", "stats"))
    mt = st["mt"]

    def temper(y):
        y = y ^ (y >> np.uint32(11))
        y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
        y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
        return y ^ (y >> np.uint32(18))

    for i, s in enumerate(seeds):
        cp = random.Random(s).getstate()[1]
        assert np.array_equal(mt[i], np.array(cp[:624], np.uint32)), f"seed {s}"
        assert int(st["stats"][13, i]) == cp[624] == 624
        assert np.array_equal(temper(_twist(mt[i])), d["words"][i][:624]), f"seed {s}"
    # and the engine draws from it: reset + a few steps against the oracle
    b.reset()
    ob = O.OracleBatch(len(seeds), seeds)
    ob.reset()
    acts = np.full((30, len(seeds)), 2, np.uint8)
    ref = ob.rollout(acts)
    for t in range(30):
        obs, rew, done = b.step(torch.as_tensor(acts[t], device=b.device))
        assert np.array_equal(obs.cpu().numpy().view(np.uint32).T, ref["obs"][t]), t
    fin = b.get_state(("mt", "stats"))
    for i in range(len(seeds)):
        assert int(fin["stats"][13, i]) == ob.envs[i].rng.index
        assert np.array_equal(fin["mt"][i], np.ctypeslib.as_array(ob.envs[i].rng.mt))


@pytest.mark.parametrize("name", sorted(CRAFTED))
def test_hip_crafted(name):
    meta, arrs = CRAFTED[name]
    replay_crafted(HipAdapter, name, meta, arrs)


@pytest.mark.parametrize("name", sorted(ROLL))
def test_hip_uniform_rollouts(name):
    meta, arrs = ROLL[name]
    replay_rollout(HipAdapter, name, meta, arrs)


@pytest.mark.parametrize("name", sorted(GREEDY))
def test_hip_greedy_rollouts(name):
    meta, arrs = GREEDY[name]
    replay_rollout(HipAdapter, name, meta, arrs)


def _oracle_vs_hip(n, steps, kw, seed_base=7, action_seed=99, autoreset="none"):
    """Full-size bit-exact check against the C oracle on splitmix64 actions."""
    G = _engine()
    b = G.TetrisBatch(n, autoreset=autoreset, seeds=[seed_base + e for e in range(n)], **kw)
    b.reset()
    ob = O.OracleBatch(n, [seed_base + e for e in range(n)], **kw)
    ob.reset()
    acts = O.splitmix64_actions(action_seed, 0, steps, n)
    ref = ob.rollout(acts)
    for t in range(steps):
        a = b.gen_actions(t, action_seed)
        assert np.array_equal(a.cpu().numpy(), acts[t])
        obs, rew, done = b.step(a, obs="packed")
        assert np.array_equal(rew.cpu().numpy(), ref["reward"][t]), f"reward t={t}"
        d = done.cpu().numpy()
        assert np.array_equal(d.astype(np.uint8), ref["done"][t]), f"done t={t}"
        assert np.array_equal(obs.cpu().numpy().view(np.uint32).T, ref["obs"][t]), f"obs t={t}"
        if autoreset == "none" and d.any():
            b.reset(torch.as_tensor(d.astype(np.uint8), device=b.device))
    return ref


@pytest.mark.parametrize("kw", [dict(), dict(advanced_clears=True, penalise_holes_increase=True,
                                             penalise_height_increase=True)])
def test_hip_vs_oracle_full_size(kw):
    """N = 65,536 (BASELINE configs C3/C4) bit-exact vs the oracle, 48 steps."""
    _oracle_vs_hip(65536, 48, dict(width=10, height=20, **kw))


def test_hip_vs_oracle_lock_delay_odd_board():
    _oracle_vs_hip(4096, 120, dict(width=9, height=15, lock_delay=2, step_reset=True,
                                   penalise_height=True, penalise_holes=True, reward_step=True))


@pytest.mark.parametrize("W,H", [(4, 4), (32, 28), (5, 27), (31, 6)])
def test_hip_vs_oracle_extreme_boards(W, H):
    """The smallest and largest boards st_create accepts (4..32 x 4..28) and
    lopsided ones, on the generic (runtime W, H) kernel: bit-exact against
    the oracle over 300 steps with same-step auto-reset (a 4x4 board dies
    every few steps, so resets and spawns into a full board dominate)."""
    _oracle_vs_hip(1024, 300, dict(width=W, height=H, advanced_clears=True, penalise_height=True,
                                   penalise_holes_increase=True), autoreset="same_step")


def test_same_step_autoreset_equals_explicit_reset():
    """autoreset='same_step' == 'none' + reset(done) on the same stream."""
    G = _engine()
    n, T = 2048, 300
    a = G.TetrisBatch(n, autoreset="none", seeds=range(n), penalise_holes_increase=True)
    b = G.TetrisBatch(n, autoreset="same_step", seeds=range(n), penalise_holes_increase=True)
    a.reset()
    b.reset()
    for t in range(T):
        act = a.gen_actions(t, 5)
        oa, ra, da = a.step(act)
        oa, ra, da = oa.clone(), ra.clone(), da.clone()
        ob, rb, db = b.step(act)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        if da.any():
            ia = a.info_tensors()
            ib = b.info_tensors()
            dd = da
            assert torch.equal(ia["score"][dd], ib["ep_score"][dd])
            assert torch.equal(ia["time"][dd], ib["ep_time"][dd])
            assert torch.equal(ia["lines_cleared"][dd], ib["ep_lines"][dd])
            a.reset(da.to(torch.uint8))
    sa, sb = a.get_state(), b.get_state()
    for k in ("board", "piece", "mt"):
        assert np.array_equal(sa[k], sb[k]), k
    assert np.array_equal(sa["stats"][:14], sb["stats"][:14])


def test_reset_zeroes_host_written_holes_and_height():
    """Default scoring flags (the kernel that never loads the old holes /
    piece_height rows): host-written nonzero holes and heights survive locks
    the reference's way (holes recounted at every lock, :278/:284; height
    untouched, :289-292) and a same-step reset zeroes both like clear() (:308,
    :310), i.e. exactly as 'none' + an explicit reset on the same stream."""
    G = _engine()
    n, T = 1024, 400
    a = G.TetrisBatch(n, autoreset="none", seeds=range(n))
    b = G.TetrisBatch(n, autoreset="same_step", seeds=range(n))
    a.reset()
    b.reset()
    rng = np.random.default_rng(7)
    st = a.get_state(("stats",))["stats"]
    st[3] = rng.integers(0, 50, n)
    st[4] = rng.integers(1, 20, n)
    a.set_state(stats=st)
    b.set_state(stats=st.copy())
    died, mixed = 0, False
    for t in range(T):
        act = a.gen_actions(t, 11)
        oa, ra, da = a.step(act)
        oa, ra, da = oa.clone(), ra.clone(), da.clone()
        ob, rb, db = b.step(act)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        if da.any():
            died += int(da.sum())
            a.reset(da.to(torch.uint8))
        sa, sb = a.get_state(("stats",))["stats"], b.get_state(("stats",))["stats"]
        assert np.array_equal(sa[:14], sb[:14]), t
        # host-written heights kept through locks beside envs a reset zeroed
        mixed |= bool((sb[4] != 0).any() and (sb[4] == 0).any())
    assert died > 0 and mixed


def test_sharding_invariance():
    """Envs keyed by global index: one batch of N == two shards of N/2."""
    G = _engine()
    n, T, seed = 1000, 200, 31
    full = G.TetrisBatch(n, autoreset="same_step", seeds=[seed + e for e in range(n)])
    h = n // 2
    sh = [G.TetrisBatch(h, autoreset="same_step", seeds=[seed + off + e for e in range(h)])
          for off in (0, h)]
    for b in [full] + sh:
        b.reset()
    for t in range(T):
        of, rf, df = full.step(full.gen_actions(t, 77))
        parts = [b.step(b.gen_actions(t, 77, global_offset=off))
                 for b, off in zip(sh, (0, h))]
        assert torch.equal(rf, torch.cat([p[1] for p in parts]))
        assert torch.equal(df, torch.cat([p[2] for p in parts]))
        assert torch.equal(of, torch.cat([p[0] for p in parts], dim=1))


def test_fused_f32_obs_equals_unpacked():
    G = _engine()
    for (W, H, n) in [(10, 20, 1000), (7, 13, 333), (12, 26, 64)]:
        b = G.TetrisBatch(n, width=W, height=H, seeds=range(n), autoreset="same_step")
        b.reset()
        for t in range(40):
            f32, rew, done = b.step(b.gen_actions(t, 3), obs="f32")
            ref = b.obs_to_f32(b.obs)
            assert torch.equal(f32, ref), (W, H, t)
            bits = ((b.obs.cpu().numpy().view(np.uint32).T[:, :, None] >> np.arange(H)) & 1)
            assert np.array_equal(ref.cpu().numpy(), bits.astype(np.float32))


def test_grayscale_kernel_matches_reference_images():
    G = _engine()
    d = np.load(f"{GOLDEN}/grayscale.npz")
    for i, (W, H) in enumerate(d["dims"]):
        if W < 4 or H < 4:
            continue
        b = G.TetrisBatch(1, width=int(W), height=int(H), seeds=[0])
        cols = (d["boards"][i][:W, :H].astype(np.uint64) << np.arange(H, dtype=np.uint64)).sum(1)
        packed = torch.as_tensor(cols.astype(np.uint32).view(np.int32)[:, None].copy(),
                                 device=b.device)
        for size, key in ((84, "g84"), (160, "g160")):
            g = b.grayscale(packed, size, 1)[0, :, :, 0].cpu().numpy()
            assert np.array_equal(g, d[key][i].astype(np.float32)), (i, size)
            g3 = b.grayscale(packed, size, 3, as_u8=True)[0].cpu().numpy()
            assert np.array_equal(g3, np.repeat(d[key][i][:, :, None], 3, axis=2)), (i, size)


def _image_np(cols, W, H, size):
    """convert_grayscale (tetris_env.py:76-114) per env from packed columns
    [n][W] (the closed form pinned by test_grayscale_kernel_matches_reference_images)."""
    lim = max(W, H)
    gap = size // 100 + 1
    blk = (size - 2 * gap) // lim - gap
    pitch = blk + gap
    pr, pc = (size - (gap + pitch * H)) // 2, (size - (gap + pitch * W)) // 2
    r = np.arange(size) - pr
    c = np.arange(size) - pc
    rin = (r >= 0) & (r < gap + pitch * H)
    cin = (c >= 0) & (c < gap + pitch * W)
    rcell = rin & (r % pitch >= gap)
    ccell = cin & (c % pitch >= gap)
    y = np.where(rcell, r // pitch, 0)
    x = np.where(ccell, c // pitch, 0)
    cols = np.asarray(cols, np.uint64)
    bits = (cols[:, x][:, None, :] >> y.astype(np.uint64)[None, :, None]) & np.uint64(1)  # [n][r][c]
    img = np.where(rin[:, None] & cin[None, :], 128, 0)[None].repeat(len(cols), 0)
    img = np.where((rcell[:, None] & ccell[None, :])[None] & (bits == 1), 190, img)
    return img


@pytest.mark.parametrize("n", [1, 17, 1000])
def test_image_kernels_ragged_batches(n):
    """st_grayscale / st_obs_to_f32 over ragged batches, every size / channel
    / dtype path: the sweep-order image kernel (a wave's 64 chunks within two
    envs) and the per-block one it falls back to (tiny images: 4x4 boards at
    sizes 12-18, and u8 totals that are not a multiple of 16 B)."""
    G = _engine()
    for (W, H, sizes) in ((10, 20, (84, 160, 50)), (7, 13, (84, 160, 50)), (4, 4, (12, 16, 18))):
        b = G.TetrisBatch(n, width=W, height=H, seeds=range(n), autoreset="same_step")
        b.reset()
        for t in range(30):
            b.step(b.gen_actions(t, 9))
        cols = b.obs.cpu().numpy().view(np.uint32).T.astype(np.uint64)   # [n][W]
        f32 = b.obs_to_f32().cpu().numpy()
        ref = ((cols[:, :, None] >> np.arange(H, dtype=np.uint64)) & 1).astype(np.float32)
        assert np.array_equal(f32, ref), (W, H)
        for size in sizes:
            exp = _image_np(cols, W, H, size)
            for ch in (1, 3):
                for u8 in (False, True):
                    g = b.grayscale(b.obs, size, ch, as_u8=u8).cpu().numpy()
                    assert g.shape == (n, size, size, ch)
                    assert np.array_equal(g, np.repeat(exp[..., None], ch, axis=3).astype(g.dtype)), \
                        (W, H, size, ch, u8)


# ---------------------------------------------------------------- single-env surface
@pytest.mark.parametrize("name", ["default", "adv_holes_height", "high_height_holes", "lock2_reset"])
@pytest.mark.parametrize("rng", ["private", "global"])
def test_single_env_surface_vs_reference(name, rng):
    """TetrisEnv (reference surface): obs float32 arrays, reward values AND
    Python types, done, info dict -- vs the reference's recorded env 0."""
    G = _engine()
    sets = GREEDY if name in GREEDY else ROLL
    meta, arrs = sets[name]
    kw = dict(meta["cfg"])
    seed = meta["seed_base"]
    env = G.TetrisEnv(rng=rng, seed=seed if rng == "private" else None, **kw)
    if rng == "global":
        random.seed(seed)
    obs = env.reset()
    assert obs.dtype == np.float32 and not obs.any()
    W = kw.get("width", 10)
    H = kw.get("height", 20)
    types = {0: int, 1: np.int64, 2: float, 3: np.float64}
    for t in range(min(300, arrs["actions"].shape[0])):
        o, r, d, info = env.step(int(arrs["actions"][t, 0]))
        assert o.shape == (W, H) and o.dtype == np.float32
        bits = ((arrs["obs"][t, 0][:, None] >> np.arange(H)) & 1).astype(np.float32)
        assert np.array_equal(o, bits), t
        assert r == arrs["reward"][t, 0] and type(r) is types[int(arrs["rtype"][t, 0])], \
            (t, r, type(r), arrs["rtype"][t, 0])
        assert d == bool(arrs["done"][t, 0])
        assert info["time"] == arrs["time"][t, 0] and info["score"] == arrs["score"][t, 0]
        assert info["holes"] == arrs["holes"][t, 0] and info["deaths"] == arrs["deaths"][t, 0]
        assert info["lines_cleared"] == arrs["lines"][t, 0]
        assert list(info["statistics"].values()) == list(arrs["counts"][t, 0])
        assert info["current_piece"] == G.SHAPE_NAMES[int(arrs["piece"][t, 0]) & 7]
        if d:
            env.reset()
    if rng == "global":
        # the global MT state must be where the reference leaves it
        ob = O.OracleBatch(1, [seed], **kw)
        ob.reset()
        ob.rollout(arrs["actions"][:min(300, arrs["actions"].shape[0]), :1])
        st = random.getstate()[1]
        mt = np.ctypeslib.as_array(ob.envs[0].rng.mt)
        assert np.array_equal(np.asarray(st[:624], np.uint32), mt)
    env.close()


def test_single_env_global_rng_with_user_draws():
    """TetrisEnv(rng='global') while the program also uses `random` between
    steps (random(), randint(), a re-seed mid-run): every step and the final
    random.getstate() equal the oracle driven by one shared CPython state --
    the reference's behaviour, where the env's draws and the user's
    interleave on the global MT (tetris_env.py:187)."""
    G = _engine()
    kw = dict(advanced_clears=True, penalise_holes_increase=True)
    acts = np.random.default_rng(5).integers(0, 7, 400)

    def user(t, rnd):
        if t % 37 == 5:
            rnd.random()
        if t % 53 == 7:
            rnd.randint(0, 9)
        if t == 200:
            rnd.seed(99)

    random.seed(11)
    env = G.TetrisEnv(rng="global", **kw)
    env.reset()
    got = []
    for t, a in enumerate(acts):
        user(t, random)
        o, r, d, _ = env.step(int(a))
        got.append((o.copy(), r, d))
        if d:
            env.reset()
    final = random.getstate()
    env.close()

    R = random.Random(11)  # the same program on the oracle, one CPython state throughout
    ob = O.OracleBatch(1, [0], **kw)

    def oracle_call(fn):
        mt, idx = R.getstate()[1][:624], R.getstate()[1][624]
        ob.envs[0].rng.mt[:] = mt
        ob.envs[0].rng.index = idx
        out = fn()
        old = R.getstate()
        R.setstate((old[0], tuple(int(x) for x in ob.envs[0].rng.mt) + (int(ob.envs[0].rng.index),), old[2]))
        return out
    oracle_call(lambda: ob.reset(0))
    for t, a in enumerate(acts):
        user(t, R)
        o, r, d, _ = oracle_call(lambda: ob.step_one(0, int(a)))
        assert np.array_equal(got[t][0], o.astype(np.float32)), t
        assert got[t][1] == r and got[t][2] == d, t
        if d:
            oracle_call(lambda: ob.reset(0))
    assert final == R.getstate()


def test_export_env_any_env_every_part():
    """st_export_env on envs 0, 37 and n-1 of a running batch, all parts: the
    record equals the step's outputs, the counters and MT state that
    st_mt_sync then produces (the export itself changes nothing), and the
    float32 obs equals the packed words unpacked; parts not asked for stay
    untouched; bad arguments are refused."""
    G = _engine()
    from gym_simpletetris_amd import _lib as C
    n, W, H = 300, 10, 20
    b = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", advanced_clears=True)
    b.reset()
    for t in range(200):
        o, r, d = b.step(b.gen_actions(t, 5))
    L, ctx = b._L, b._ctx
    sp = ctypes.c_void_p(torch.cuda.current_stream(b.device).cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    nw = L.st_export_words(W, H)
    assert nw == W + 2 + C.NSTAT + C.MT_N + W * H
    recs = {}
    for env in (0, 37, n - 1):
        rec = torch.zeros(nw, dtype=torch.int32, device=b.device)
        C.check(L.st_export_env(ctx, env, P(o), P(r), P(d), C.EXPORT_MT | C.EXPORT_OBS_F32, P(rec), sp))
        recs[env] = rec.cpu().numpy()
    words = o.cpu().numpy().view(np.uint32)
    rew, done = r.cpu().numpy(), d.cpu().numpy()
    st = b.get_state(("stats", "mt"))  # st_mt_sync: the canonical form the export computed read-only
    m = W + 2 + C.NSTAT
    for env, rec in recs.items():
        assert np.array_equal(rec[:W].view(np.uint32), words[:, env]), env
        assert rec[W] == rew[env] and rec[W + 1] == int(done[env]), env
        assert np.array_equal(rec[W + 2:m], st["stats"][:, env]), env
        assert np.array_equal(rec[m:m + C.MT_N].view(np.uint32), st["mt"][env]), env
        f32 = rec[m + C.MT_N:].view(np.float32).reshape(W, H)
        bits = ((words[:, env][:, None].astype(np.uint64) >> np.arange(H, dtype=np.uint64)) & 1).astype(np.float32)
        assert np.array_equal(f32, bits), env
    rec = torch.full((nw,), -7, dtype=torch.int32, device=b.device)
    C.check(L.st_export_env(ctx, 5, P(o), P(r), P(d), 0, P(rec), sp))
    h = rec.cpu().numpy()
    assert (h[m:] == -7).all() and np.array_equal(h[:W].view(np.uint32), words[:, 5])
    for env, parts in ((n, 0), (-1, 0), (0, 4)):
        with pytest.raises(C.StError):
            C.check(L.st_export_env(ctx, env, P(o), P(r), P(d), parts, P(rec), sp))
    b.close()


def test_single_env_errors_and_render():
    G = _engine()
    env = G.make("SimpleTetris-v0", rng="private", seed=3)
    with pytest.raises(AttributeError):
        env.step(0)
    env.reset()
    with pytest.raises(KeyError):
        env.step(7)
    for bad in (2.5, -1, float("nan"), "2", None):  # not keys of value_action_map
        with pytest.raises(KeyError):
            env.step(bad)
    env.step(2.0)  # value_action_map[2.0] is value_action_map[2]
    env.step(np.int8(3))
    env.step(True)  # True == 1 and hashes alike: right
    img = env.render("rgb_array")
    assert img.shape == (160, 160, 3) and img.dtype == np.uint8
    assert set(np.unique(img)) <= {0, 128, 190} and (img == 190).any()  # piece drawn
    g = G.make("SimpleTetris-v0", obs_type="grayscale", extend_dims=True, rng="private")
    o = g.reset()
    assert o.shape == (84, 84, 1) and o.dtype == np.float32
    o, r, d, info = g.step(2)
    assert set(np.unique(o)) <= {0.0, 128.0, 190.0}
    rgb = G.make("SimpleTetris-v0", obs_type="rgb", rng="private")
    rgb.reset()
    o, *_ = rgb.step(6)
    assert o.shape == (84, 84, 3)


@pytest.mark.parametrize("name", sorted(RENDER))
def test_render_and_image_obs_vs_reference(name):
    """render_packed() (engine.render(), tetris_env.py:317-321), the
    160x160x3 render('rgb_array') frame (:458-462) and the 'grayscale' /
    'rgb' observations (:413-433) bit for bit against the reference's own
    outputs along the same games (tests/golden/render.npz)."""
    G = _engine()
    meta, arrs = RENDER[name]
    envs = {ot: G.TetrisEnv(obs_type=ot, rng="private", seed=meta["seed"], **meta["cfg"])
            for ot in ("ram", "grayscale", "rgb")}
    for env in envs.values():
        env.reset()
    k = 0
    for t, a in enumerate(arrs["actions"]):
        obs = {}
        for ot, env in envs.items():
            o, r, d, info = env.step(int(a))
            obs[ot] = o
            if d:
                env.reset()
        if t in meta["at"]:
            e = envs["ram"]
            packed = e.engine.render_packed().cpu().numpy().view(np.uint32)[:, 0]
            assert np.array_equal(packed, arrs["render"][k]), (name, t)
            img = e.render("rgb_array")
            assert img.dtype == np.uint8 and img.shape == (160, 160, 3)
            assert np.array_equal(img, np.repeat(arrs["rgb160"][k][:, :, None], 3, axis=2)), (name, t)
            g = obs["grayscale"]
            assert g.dtype == np.float32 and g.shape == (84, 84)
            assert np.array_equal(g, arrs["gray84"][k].astype(np.float32)), (name, t)
            c = obs["rgb"]
            assert c.dtype == np.float32 and c.shape == (84, 84, 3)
            assert np.array_equal(c, np.repeat(arrs["gray84"][k][:, :, None], 3, axis=2).astype(np.float32))
            k += 1
    assert k == len(meta["at"])
    for env in envs.values():
        env.close()


def test_vec_env_surface():
    G = _engine()
    v = G.make("SimpleTetrisVec-v0", num_envs=256, seed=11, advanced_clears=True)
    o = v.reset()
    assert o.shape == (256, 10, 20) and o.dtype == torch.float32 and not o.any()
    for t in range(100):
        o, r, d, info = v.step(torch.randint(0, 7, (256,), dtype=torch.uint8, device=v.device))
        assert o.shape == (256, 10, 20) and r.dtype == torch.int32 and d.dtype == torch.bool
    assert info["time"].shape == (256,)
    assert int(info["deaths"].sum()) > 0
    # an info kept past later steps still describes its own step
    # (hard drops: some envs finish an episode in the kept step)
    _, _, kd, kept = v.step(torch.full((256,), 2, dtype=torch.uint8, device=v.device))
    kd = kd.clone()
    live = {k: x.clone() for k, x in v.engine.info_tensors().items()}   # the state right now
    for _ in range(3):
        v.step(torch.full((256,), 2, dtype=torch.uint8, device=v.device))
    for k in ("time", "score", "holes", "deaths", "statistics"):
        assert torch.equal(kept[k], live[k]), k
    # ep_*: the episode finished in that step where the env was reset in it,
    # else 0 (the engine's EP rows keep the last finished episode)
    assert kd.any()
    for k in ("ep_time", "ep_score", "ep_lines", "ep_holes"):
        assert torch.equal(kept[k], torch.where(kd, live[k], torch.zeros_like(live[k]))), k
    assert not torch.equal(v.engine.info_tensors()["time"], live["time"])


def test_vec_env_unvalidated_actions():
    """validate_actions=False: no check (no sync); an out-of-range action acts
    as idle (action 6), in-range ones as usual.  The default ('async': the
    step kernel's own check) raises KeyError at the next step; True raises
    before the step."""
    G = _engine()
    n = 512
    a = G.TetrisVecEnv(n, seed=4, validate_actions=False, obs_format="packed")
    b = G.TetrisVecEnv(n, seed=4, obs_format="packed")
    c = G.TetrisVecEnv(n, seed=4, obs_format="packed", validate_actions=True)
    assert b.engine.validate_actions == "async"
    a.reset()
    b.reset()
    c.reset()
    g = torch.Generator(device="cpu").manual_seed(0)
    for t in range(60):
        acts = torch.randint(0, 10, (n,), dtype=torch.uint8, generator=g).to(a.device)
        oa, ra, da, _ = a.step(acts)
        ok = torch.where(acts > 6, torch.full_like(acts, 6), acts)
        ob, rb, db, _ = b.step(ok)
        oc, rc, dc, _ = c.step(ok)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        assert torch.equal(oa, oc) and torch.equal(ra, rc) and torch.equal(da, dc), t
    b.check_actions()  # nothing flagged
    b.step(torch.full((n,), 7, dtype=torch.uint8, device=b.device))  # flagged by the kernel, no sync
    with pytest.raises(KeyError):
        b.check_actions()
    with pytest.raises(KeyError):
        c.step(torch.full((n,), 7, dtype=torch.uint8, device=c.device))
    for v in (a, b, c):
        v.close()


def test_async_action_check():
    """validate_actions='async': the step kernel flags an out-of-range
    action (st_set_action_flag) without a sync or an extra launch; the
    KeyError comes at the next step after the flag is seen (or from
    check_actions()), and the steps equal unvalidated ones.  The same for
    st_rollout (a bad action in any of its steps), and for non-uint8 device
    tensors (int64 -1 / 263 / 256 and non-integral floats, which a uint8
    cast would wrap into range, are mapped to 255 on the device first).
    st_check_actions (the stand-alone check) itself: every byte position,
    the unaligned / ragged tail path, values 7 and 255."""
    G = _engine()
    from gym_simpletetris_amd import _lib as C
    n = 1000
    a = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions="async")
    b = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=False)
    a.reset()
    b.reset()
    for t in range(20):
        acts = b.gen_actions(t, 3).clone()
        oa, ra, da = a.step(acts)
        ob, rb, db = b.step(acts)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    a.check_actions()  # nothing flagged
    bad = b.gen_actions(99, 3).clone()
    bad[617] = 9
    a.step(bad)  # no sync, no error yet
    torch.cuda.synchronize()
    with pytest.raises(KeyError):
        a.step(b.gen_actions(100, 3))
    a.step(b.gen_actions(101, 3))  # the flag was cleared
    a.check_actions()
    a.step(bad)
    with pytest.raises(KeyError):
        a.check_actions()
    # no sync on the async path: the kernel's flag is the only check
    assert a._flag_dev is not None
    # st_rollout: a bad action in a later step of the launch is flagged
    ra = torch.stack([b.gen_actions(200 + t, 3).clone() for t in range(5)])
    a.rollout(ra)
    a.check_actions()
    ra[3, 999] = 7
    a.rollout(ra)
    with pytest.raises(KeyError):
        a.check_actions()
    # wider dtypes: values a uint8 cast would wrap into 0..6
    for badv, dt in ((256, torch.int64), (-1, torch.int64), (263, torch.int32), (2.5, torch.float32),
                     (-1, torch.int8), (127, torch.int8), (-1, torch.int16), (256, torch.int16)):
        x = b.gen_actions(300, 3).to(dt)
        x[5] = badv
        a.step(x)
        with pytest.raises(KeyError):
            a.check_actions()
    for dt in (torch.float64, torch.int8, torch.int16):  # in-range values of every dtype pass (2.0 == 2)
        x = b.gen_actions(301, 3).to(dt)
        a.step(x)
        a.check_actions()
    # the kernel on its own
    L = a._L
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    flag = torch.zeros(1, dtype=torch.int32, device=a.device)
    buf = torch.zeros(4096 + 16, dtype=torch.uint8, device=a.device)
    for length, off in ((4096, 0), (4096, 1), (37, 3), (1, 0)):
        for pos in sorted({0, length // 2, length - 1}):
            for v in (6, 7, 255):
                buf.zero_()
                flag.zero_()
                buf[off + pos] = v
                C.check(L.st_check_actions(ctypes.c_void_p(buf.data_ptr() + off), length,
                                           ctypes.c_void_p(flag.data_ptr()), sp))
                assert int(flag.item()) == (1 if v > 6 else 0), (length, off, pos, v)
    a.close()
    b.close()


@pytest.mark.parametrize("scoring", ["penalties", "default"])
@pytest.mark.parametrize("autoreset", ["same_step", "none"])
@pytest.mark.parametrize("board", [(10, 20), (9, 15)])
def test_rollout_equals_steps(autoreset, board, scoring):
    """st_rollout(K) == K x st_step, bit-exact, outputs and final state.
    "default" scoring (no holes term in the reward): the rollout counts holes
    only where it reads them (a death, the final state), st_step at every
    lock -- the final holes counters and the episode counters must agree."""
    G = _engine()
    W, H = board
    n, K = 1000, 150
    kw = dict(width=W, height=H, lock_delay=1, step_reset=True)
    if scoring == "penalties":
        kw.update(penalise_holes_increase=True, advanced_clears=True, penalise_height_increase=True)
    a = G.TetrisBatch(n, autoreset=autoreset, seeds=[3 + e for e in range(n)], **kw)
    b = G.TetrisBatch(n, autoreset=autoreset, seeds=[3 + e for e in range(n)], **kw)
    a.reset()
    b.reset()
    acts = torch.stack([a.gen_actions(t, 11).clone() for t in range(K)])
    for obs_mode in ("packed", "f32"):
        ro, rr, rd = b.rollout(acts, obs=obs_mode)
        for t in range(K):
            so, sr, sd = a.step(acts[t], obs=obs_mode)
            assert torch.equal(so, ro[t]), (obs_mode, t)
            assert torch.equal(sr, rr[t]) and torch.equal(sd, rd[t]), (obs_mode, t)
        sa, sb = a.get_state(), b.get_state()
        for k in sa:
            assert np.array_equal(sa[k], sb[k]), (obs_mode, k)


@pytest.mark.parametrize("autoreset", ["same_step", "none"])
def test_rollout_short_launches_queue_edges(autoreset):
    """The three-wave st_rollout's piece queue and action ring at their edges:
    launches of 1, 2, 3 and 5 steps (the action ring's first four rows come
    from the draw wave's initial loads; the logic wave's first waits have
    their own thresholds), hard drops on half the steps (a lock at most
    steps: the queue drained two pieces deep while the draw wave lags), and
    a state read-back in the middle (st_mt_sync: every env restarts without
    a preview, so the first rollout after it draws q0 and q1 at its start).
    Outputs and final state == the same steps through st_step."""
    G = _engine()
    n = 1000
    kw = dict(width=10, height=20, advanced_clears=True, penalise_holes_increase=True)
    a = G.TetrisBatch(n, autoreset=autoreset, seeds=[40 + e for e in range(n)], **kw)
    b = G.TetrisBatch(n, autoreset=autoreset, seeds=[40 + e for e in range(n)], **kw)
    a.reset()
    b.reset()
    lengths = [1, 2, 3, 5, 1, 1, 4, 3, 2, 5, 1]
    T = 2 * sum(lengths)
    acts = torch.stack([a.gen_actions(t, 23).clone() for t in range(T)])
    acts[::2] = 2  # hard drops
    t = 0
    for rep in range(2):
        for k in lengths:
            ro, rr, rd = a.rollout(acts[t:t + k], obs="packed")
            for j in range(k):
                so, sr, sd = b.step(acts[t + j], obs="packed")
                assert torch.equal(so, ro[j]), (rep, t, j)
                assert torch.equal(sr, rr[j]) and torch.equal(sd, rd[j]), (rep, t, j)
            t += k
        sa, sb = a.get_state(), b.get_state()  # synced: no preview in either afterwards
        for key in sa:
            assert np.array_equal(sa[key], sb[key]), (rep, key)


def test_rollout_vs_oracle_full_size():
    """N = 65,536, K = 32 steps in one launch vs the C oracle."""
    G = _engine()
    n, K, seed_a = 65536, 32, 99
    kw = dict(width=10, height=20)
    b = G.TetrisBatch(n, autoreset="same_step", seeds=[7 + e for e in range(n)], **kw)
    b.reset()
    ob = O.OracleBatch(n, [7 + e for e in range(n)], **kw)
    ob.reset()
    acts = O.splitmix64_actions(seed_a, 0, K, n)
    ref = ob.rollout(acts)
    obs, rew, done = b.rollout(torch.as_tensor(acts, device=b.device))
    assert np.array_equal(rew.cpu().numpy(), ref["reward"])
    assert np.array_equal(done.cpu().numpy().astype(np.uint8), ref["done"])
    assert np.array_equal(obs.cpu().numpy().view(np.uint32).transpose(0, 2, 1), ref["obs"])


def _untemper(y):
    """Inverse of MT19937 tempering (so crafted state words produce chosen outputs)."""
    def undo_r(y, s):
        x = y
        for _ in range(32 // s + 1):
            x = y ^ (x >> s)
        return x & 0xFFFFFFFF

    def undo_l(y, s, m):
        x = y
        for _ in range(32 // s + 1):
            x = y ^ ((x << s) & m)
        return x & 0xFFFFFFFF
    y = undo_r(y, 18)
    y = undo_l(y, 15, 0xEFC60000)
    y = undo_l(y, 7, 0x9D2C5680)
    return undo_r(y, 11)


@pytest.mark.parametrize("mode", ["step", "rollout"])
def test_long_rejection_runs_and_twists(mode):
    """Crafted MT states: draws that reject 10 words in a row (the second
    half of the 16-word prefetch), 20 (past it: the dependent-load loop), and
    states 1-3 words from a generation's end whose successor is not built
    (host-written state: finished cooperatively), against the oracle."""
    G = _engine()
    n, T = 64, 40
    b = G.TetrisBatch(n, autoreset="same_step", seeds=range(n))
    b.reset()
    ob = O.OracleBatch(n, list(range(n)))
    ob.reset()
    st = b.get_state(("mt", "stats"))
    mt, stats = st["mt"].copy(), st["stats"].copy()
    rej, acc = _untemper(0xFFFFFFFF), _untemper(0)
    for i in range(n):
        idx = int(stats[13, i])
        if i % 4 == 0 and idx + 21 <= 624:          # 20 rejections, then accept
            mt[i, idx:idx + 20] = rej
            mt[i, idx + 20] = acc
        elif i % 4 == 1:                             # next draws cross the twist
            idx = 621 + (i % 3)
            stats[13, i] = idx
        elif i % 4 == 2 and idx + 41 <= 624:         # two long runs back to back
            mt[i, idx:idx + 18] = rej
            mt[i, idx + 18] = acc
            mt[i, idx + 19:idx + 40] = rej
            mt[i, idx + 40] = acc
        elif i % 4 == 3 and idx + 11 <= 624:         # 10 rejections: the second prefetched half
            mt[i, idx:idx + 10] = rej
            mt[i, idx + 10] = acc
        e = ob.envs[i]
        for k in range(624):
            e.rng.mt[k] = int(mt[i, k])
        e.rng.index = int(stats[13, i])
    b.set_state(mt=mt, stats=stats)
    acts = np.full((T, n), 2, np.uint8)              # hard drops: a lock every step
    acts[::3] = O.splitmix64_actions(5, 0, T, n)[::3]
    ref = ob.rollout(acts)
    if mode == "step":
        for t in range(T):
            obs, rew, done = b.step(torch.as_tensor(acts[t], device=b.device))
            assert np.array_equal(rew.cpu().numpy(), ref["reward"][t]), t
            assert np.array_equal(obs.cpu().numpy().view(np.uint32).T, ref["obs"][t]), t
    else:
        obs, rew, done = b.rollout(torch.as_tensor(acts, device=b.device))
        assert np.array_equal(rew.cpu().numpy(), ref["reward"])
        assert np.array_equal(done.cpu().numpy().astype(np.uint8), ref["done"])
        assert np.array_equal(obs.cpu().numpy().view(np.uint32).transpose(0, 2, 1), ref["obs"])
    fin = b.get_state(("mt", "stats"))
    for i in range(n):
        assert int(fin["stats"][13, i]) == ob.envs[i].rng.index, i
        assert np.array_equal(fin["mt"][i], np.ctypeslib.as_array(ob.envs[i].rng.mt)), i


def test_mt_generations_across_steps():
    """Lock every step for ~2.5 MT generations: the next generation is built
    a block per draw into a second buffer and switched to at index 624, so
    states between steps carry engine bits; st_mt_sync must restore CPython's
    exact state at any point, and syncing mid-run (which restarts the next
    generation's progress) must not change what follows."""
    import ctypes
    from gym_simpletetris_amd import _lib as C
    G = _engine()
    n, T, chunk = 256, 1200, 100
    seeds = [11 + e for e in range(n)]
    a = G.TetrisBatch(n, autoreset="same_step", seeds=seeds)
    b = G.TetrisBatch(n, autoreset="same_step", seeds=seeds)
    a.reset()
    b.reset()
    ob = O.OracleBatch(n, seeds)
    ob.reset()
    acts = np.full((T, n), 2, np.uint8)              # hard drops: a draw every step
    acts[::4] = O.splitmix64_actions(3, 0, T, n)[::4]
    ref = ob.rollout(acts)
    saw_lazy = False
    for c0 in range(0, T, chunk):
        da = torch.as_tensor(acts[c0:c0 + chunk], device=a.device)
        oa, ra, _ = a.rollout(da)
        for t in range(c0, c0 + chunk):
            ob_, rb, _ = b.step(da[t - c0])
            assert torch.equal(ob_, oa[t - c0]) and torch.equal(rb, ra[t - c0]), t
        assert np.array_equal(ra.cpu().numpy(), ref["reward"][c0:c0 + chunk]), c0
        assert np.array_equal(oa.cpu().numpy().view(np.uint32).transpose(0, 2, 1),
                              ref["obs"][c0:c0 + chunk]), c0
        # raw (unsynced) index row of b: some envs mid-generation
        raw = torch.empty(b.stride, dtype=torch.int32, device=b.device)
        v = b._views
        C.check(b._L.st_copy(ctypes.c_void_p(raw.data_ptr()),
                             ctypes.c_void_p(v.stats + C.STAT["mt_index"] * v.stride * 4),
                             raw.numel() * 4, b._stream()))
        saw_lazy |= bool((((raw[:n].cpu().numpy() >> 20) & 1) != 0).any())   # current generation in B
        if (c0 // chunk) % 3 == 1:
            a.get_state(("mt", "stats"))                # sync a only, mid-run
    assert saw_lazy
    fa, fb = a.get_state(), b.get_state()
    for k in fa:
        assert np.array_equal(fa[k], fb[k]), k
    for i in range(n):
        assert int(fa["stats"][13, i]) == ob.envs[i].rng.index, i
        assert np.array_equal(fa["mt"][i], np.ctypeslib.as_array(ob.envs[i].rng.mt)), i


@pytest.mark.parametrize("mode", ["step", "rollout"])
def test_sync_at_generation_boundary(mode):
    """A spawn whose draw takes the generation's last word (index 623) leaves
    CPython at index 624 with the OLD words (it twists lazily); the preview
    drawn right after it starts at 624 and runs into the next generation.
    st_mt_sync must give back exactly (old words, 624), and stepping on from
    the synced state must match the oracle."""
    G = _engine()
    n = 64
    b = G.TetrisBatch(n, autoreset="same_step", seeds=range(100, 100 + n))
    b.reset()
    ob = O.OracleBatch(n, list(range(100, 100 + n)))
    ob.reset()
    st = b.get_state(("mt", "stats"))
    mt, stats = st["mt"].copy(), st["stats"].copy()
    acc = _untemper(0)                  # accepted by any randint range
    for i in range(n):
        mt[i, 623] = acc
        stats[13, i] = 623
        e = ob.envs[i]
        for k in range(624):
            e.rng.mt[k] = int(mt[i, k])
        e.rng.index = 623
    b.set_state(mt=mt, stats=stats)
    acts = np.full((1, n), 2, np.uint8)  # hard drop: every env locks and spawns
    ref = ob.rollout(acts)
    if mode == "step":
        obs, rew, _ = b.step(torch.as_tensor(acts[0], device=b.device))
        assert np.array_equal(rew.cpu().numpy(), ref["reward"][0])
    else:
        obs, rew, _ = b.rollout(torch.as_tensor(acts, device=b.device))
        assert np.array_equal(rew.cpu().numpy(), ref["reward"])
    fin = b.get_state(("mt", "stats"))
    for i in range(n):
        assert ob.envs[i].rng.index == 624
        assert int(fin["stats"][13, i]) == 624, i
        assert np.array_equal(fin["mt"][i], mt[i]), i          # the old generation's words
    acts = O.splitmix64_actions(8, 0, 80, n)
    acts[::2] = 2
    ref = ob.rollout(acts)
    for t in range(80):
        obs, rew, _ = b.step(torch.as_tensor(acts[t], device=b.device))
        assert np.array_equal(rew.cpu().numpy(), ref["reward"][t]), t
        assert np.array_equal(obs.cpu().numpy().view(np.uint32).T, ref["obs"][t]), t
    fin = b.get_state(("mt", "stats"))
    for i in range(n):
        assert int(fin["stats"][13, i]) == ob.envs[i].rng.index, i
        assert np.array_equal(fin["mt"][i], np.ctypeslib.as_array(ob.envs[i].rng.mt)), i


def test_preview_rewind_across_generations():
    """Each env's next piece is drawn one spawn ahead (the preview, kept in the
    MT word with the number c of MT words its draw consumed).  A preview whose
    draw crossed index 624 straddles two generations: st_mt_sync must give its
    words back into the previous generation's buffer.  Lock every step (hard
    drops) until such states occur, sync there, compare every env's MT state
    with CPython's (the oracle), and keep stepping: after a sync the next spawn
    draws its piece, then a new preview, and the games must not change."""
    import ctypes
    from gym_simpletetris_amd import _lib as C
    G = _engine()
    n, T = 512, 1600
    seeds = [7000 + e for e in range(n)]
    b = G.TetrisBatch(n, autoreset="same_step", seeds=seeds)
    b.reset()
    ob = O.OracleBatch(n, seeds)
    ob.reset()
    acts = np.full((T, n), 2, np.uint8)              # hard drops: a draw every step
    acts[::5] = O.splitmix64_actions(11, 0, T, n)[::5]
    raw = torch.empty(b.stride, dtype=torch.int32, device=b.device)
    v = b._views
    syncs, stop, boundary = 0, T, 0
    for t in range(T):
        if t >= stop:
            break
        o, r, _ = b.step(torch.as_tensor(acts[t], device=b.device))
        ref = ob.rollout(acts[t:t + 1])
        assert np.array_equal(r.cpu().numpy(), ref["reward"][0]), t
        assert np.array_equal(o.cpu().numpy().view(np.uint32).T, ref["obs"][0]), t
        C.check(b._L.st_copy(ctypes.c_void_p(raw.data_ptr()),
                             ctypes.c_void_p(v.stats + C.STAT["mt_index"] * v.stride * 4),
                             raw.numel() * 4, b._stream()))
        w = raw[:n].cpu().numpy().astype(np.uint32)
        ok = ((w >> 24) & 1).astype(bool)
        straddle = ok & ((w & 0x3FF) < ((w >> 25) & 63))
        if straddle.any() and syncs < 3:
            st = b.get_state(("mt", "stats"))          # st_mt_sync
            for i in range(n):  # exactly random.getstate(): words and index (624 included)
                assert int(st["stats"][13, i]) == ob.envs[i].rng.index, (t, i)
                assert np.array_equal(st["mt"][i], np.ctypeslib.as_array(ob.envs[i].rng.mt)), (t, i)
                boundary += int(st["stats"][13, i]) == 624
            syncs += 1
            if syncs == 3:
                stop = t + 60                            # keep stepping past the last sync
    assert syncs == 3, "no straddling preview within the run"


def _greedy_ref(col_words, W, H, pw):
    """numpy restatement of st_policy_greedy with explore = 0 (the fixture
    generator's greedy_target / greedy_action, tests/golden/gen_golden.py,
    scores doubled to integers)."""
    board = ((np.asarray(col_words, np.uint64)[:, None] >> np.arange(H, dtype=np.uint64)) & 1).astype(bool)
    sid, rot, ax = pw & 7, (pw >> 3) & 3, (pw >> 5) & 63
    best, best_s = None, None
    for r in range(4):
        cells = O.rotate_cells(O.BASE_SHAPES[sid], r)

        def occ(x0, y0):
            for i, j in cells:
                x, y = x0 + i, y0 + j
                if y < 0:
                    continue
                if x < 0 or x >= W or y >= H or board[x, y]:
                    return True
            return False
        for x in range(-3, W + 3):
            if occ(x, 0):
                continue
            y = 0
            while not occ(x, y + 1):
                y += 1
            b, ok = board.copy(), True
            for i, j in cells:
                if 0 <= x + i < W and 0 <= y + j < H:
                    b[x + i, y + j] = True
                elif y + j < 0:
                    ok = False
            full = np.all(b, axis=0)
            keep = b[:, ~full]
            nb = np.zeros_like(b)
            nb[:, H - keep.shape[1]:] = keep
            holes = int(np.count_nonzero(nb.cumsum(axis=1) * ~nb))
            fr = np.any(nb, axis=0)
            height = H - int(np.argmax(fr)) if fr.any() else 0
            sc = 80 * int(full.sum()) - 12 * holes - 3 * height - (0 if ok else 2000)
            if best_s is None or sc > best_s:
                best_s, best = sc, (r, x)
    if best is None:
        return 2
    if rot != best[0]:
        return 4
    return 1 if ax < best[1] else (0 if ax > best[1] else 2)


def test_greedy_policy_and_clear_heavy_parity():
    """st_policy_greedy against its numpy restatement on evolving states, and
    the clear-heavy trajectory it drives against the oracle (bit-exact, with
    line clears at every count the boards produce)."""
    G = _engine()
    n, T, W, H = 128, 240, 10, 20
    seeds = [21 + e for e in range(n)]
    kw = dict(width=W, height=H, advanced_clears=True, penalise_holes_increase=True,
              penalise_height_increase=True)
    b = G.TetrisBatch(n, autoreset="same_step", seeds=seeds, **kw)
    b.reset()
    acts = np.zeros((T, n), np.uint8)
    got = []
    for t in range(T):
        if t % 40 == 7:  # the policy itself, explore off, vs numpy
            a0 = b.policy_greedy(t, seed=3, explore=0).cpu().numpy().copy()
            st = b.get_state(("board", "piece"))
            for e in range(0, n, 5):
                assert int(a0[e]) == _greedy_ref(st["board"][:, e], W, H, int(st["piece"][e])), (t, e)
        a = b.policy_greedy(t, seed=3, explore=30)
        acts[t] = a.cpu().numpy()
        o, r, d = b.step(a)
        got.append((o.cpu().numpy().view(np.uint32).T.copy(), r.cpu().numpy().copy(),
                    d.cpu().numpy().astype(np.uint8)))
    ob = O.OracleBatch(n, seeds, **kw)
    ob.reset()
    ref = ob.rollout(acts)
    # st_step on the clear-heavy trajectory (its line clears with the preview
    # and draw wave live; get_state above syncs only every 40 steps)
    for t in range(T):
        assert np.array_equal(got[t][1], ref["reward"][t]), t
        assert np.array_equal(got[t][2], ref["done"][t]), t
        assert np.array_equal(got[t][0], ref["obs"][t]), t
    c = G.TetrisBatch(n, autoreset="same_step", seeds=seeds, **kw)
    c.reset()
    obs, rew, done = c.rollout(torch.as_tensor(acts, device=c.device))
    assert np.array_equal(rew.cpu().numpy(), ref["reward"])
    assert np.array_equal(done.cpu().numpy().astype(np.uint8), ref["done"])
    assert np.array_equal(obs.cpu().numpy().view(np.uint32).transpose(0, 2, 1), ref["obs"])
    lines = c.info_tensors()["lines_cleared"].cpu().numpy()
    assert lines.sum() > n  # the point of the policy: many clears


def test_abi_error_paths():
    """The C ABI rejects bad arguments and call-order violations with codes
    and a message instead of faulting (reference: exceptions)."""
    import ctypes
    from gym_simpletetris_amd import _lib as C
    L = C.load()
    ctx = ctypes.c_void_p()
    for cfg, n in [(C.Config(3, 20, 0, 0, 0), 8), (C.Config(10, 29, 0, 0, 0), 8),
                   (C.Config(10, 20, 0, 1 << 9, 0), 8), (C.Config(10, 20, 0, 0, 7), 8),
                   (C.Config(10, 20, 40000, 0, 0), 8), (C.Config(10, 20, 0, 0, 0), 0),
                   (C.Config(10, 20, 0, 0, 0), (1 << 24) + 1)]:
        assert L.st_create(ctypes.byref(ctx), ctypes.byref(cfg), 0, n) == C.ST_EINVAL
        assert L.st_last_error()
    assert L.st_create(ctypes.byref(ctx), ctypes.byref(C.Config(10, 20, 0, 0, 0)), 99, 8) == C.ST_EINVAL
    assert L.st_create(ctypes.byref(ctx), ctypes.byref(C.Config(10, 20, 0, 0, 0)), 0, 8) == C.ST_OK
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    p = ctypes.c_void_p(d.data_ptr())
    assert L.st_step(ctx, p, None, None, None, None) == C.ST_ESTATE      # before seed/reset
    assert L.st_reset(ctx, None, None) == C.ST_ESTATE                    # before seed
    assert L.st_rollout(ctx, 4, p, None, None, None, None, None) == C.ST_ESTATE
    seeds = np.arange(8, dtype=np.uint64)
    assert L.st_seed(ctx, ctypes.c_void_p(seeds.ctypes.data), None) == C.ST_OK
    assert L.st_step(ctx, p, None, None, None, None) == C.ST_ESTATE      # before reset
    assert L.st_reset(ctx, None, None) == C.ST_OK
    assert L.st_step(ctx, None, None, None, None, None) == C.ST_EINVAL
    assert L.st_rollout(ctx, 0, p, None, None, None, None, None) == C.ST_EINVAL
    assert L.st_step(ctx, p, None, None, None, None) == C.ST_OK          # all outputs optional
    assert L.st_grayscale(ctx, p, 84, 2, 0, p, None) == C.ST_EINVAL
    assert L.st_grayscale(ctx, p, 12, 1, 0, p, None) == C.ST_EINVAL
    assert L.st_copy(None, p, 4, None) == C.ST_EINVAL
    torch.cuda.synchronize()
    assert L.st_destroy(ctx) == C.ST_OK
    assert L.st_destroy(None) == C.ST_OK


def test_wrapper_validation():
    G = _engine()
    b = G.TetrisBatch(10, seeds=range(10))
    with pytest.raises(RuntimeError):
        G.TetrisBatch(10).reset()                  # reset before seed
    with pytest.raises(ValueError):
        b.seed(range(9))
    b.reset()
    with pytest.raises(ValueError):
        b.step(np.zeros(9, np.uint8))
    with pytest.raises(ValueError):
        b.rollout(torch.zeros((3, 9), dtype=torch.uint8, device=b.device))
    with pytest.raises(ValueError):
        G.TetrisBatch(4, autoreset="sometimes")
    # actions outside value_action_map raise like the reference's KeyError
    # (tetris_env.py:245), before any uint8 cast could wrap them
    for bad in (np.full(10, 7), np.full(10, -1), np.full(10, 263)):
        with pytest.raises(KeyError):
            b.step(bad)
        with pytest.raises(KeyError):
            b.step(torch.as_tensor(bad, device=b.device))
    with pytest.raises(KeyError):
        b.step(torch.full((10,), 7, dtype=torch.uint8, device=b.device))
    with pytest.raises(KeyError):
        b.rollout(torch.full((3, 10), -1, dtype=torch.int64, device=b.device))
    # floats index value_action_map only when integral (2.0 == 2; 2.5 is no key),
    # on the numpy and the tensor path alike
    for bad in (np.full(10, 2.5), np.full(10, np.nan)):
        with pytest.raises(KeyError):
            b.step(bad)
        with pytest.raises(KeyError):
            b.step(torch.as_tensor(bad, device=b.device))
    with pytest.raises(TypeError):
        b.step(torch.zeros(10, dtype=torch.complex64, device=b.device))
    before = b.get_state()
    after = b.get_state()
    for k in before:  # rejected calls did not step
        assert np.array_equal(before[k], after[k])
    b.step(torch.arange(10, device=b.device) % 7)     # int64 device actions in range
    b.step(np.full(10, 2.0))                         # integral floats in range
    b.step(torch.full((10,), 3.0, device=b.device))
    from gym_simpletetris_amd.distributed import ShardedTetris
    sh = ShardedTetris(20, seed=5, rank=1, world=2, device=b.device)
    assert sh.engine.validate_actions == "async"  # the public step stays asynchronous
    sh.reset()
    sh.step(torch.full((10,), 9, dtype=torch.uint8, device=b.device))  # checked in the kernel
    with pytest.raises(KeyError):
        sh.engine.check_actions()
    with pytest.raises(KeyError):
        sh.step(np.full(10, 9))  # host actions: checked up front
    with pytest.raises(ValueError):
        sh.step(torch.zeros(11, dtype=torch.uint8, device=b.device))
    o, r, d = sh.step(torch.zeros(10, dtype=torch.uint8, device=b.device))
    assert o.data_ptr() == sh.buf.data_ptr()


def test_save_load_snapshot(tmp_path):
    """st_save / st_load: a snapshot restores the exact state -- replaying the
    same actions from it, in the same batch or in a fresh one seeded
    differently, reproduces every output and the final state."""
    G = _engine()
    from gym_simpletetris_amd._lib import StError
    n, K = 3000, 60
    kw = dict(advanced_clears=True, penalise_holes_increase=True, lock_delay=1, step_reset=True)
    a = G.TetrisBatch(n, autoreset="same_step", seeds=[5 + e for e in range(n)], **kw)
    a.reset()
    for t in range(40):
        a.step(a.gen_actions(t, 9))
    path = tmp_path / "snap.bin"
    snap = a.save(str(path))
    assert len(snap) == path.stat().st_size == 64 + n * 4 * (10 + 19 + 624)
    outs = []
    for t in range(K):
        outs.append(tuple(x.clone() for x in a.step(a.gen_actions(40 + t, 9))))
    fin = a.get_state()
    b = G.TetrisBatch(n, autoreset="same_step", seeds=[999] * n, **kw)
    for eng, src in ((a, snap), (b, str(path))):
        eng.load(src)
        for t in range(K):
            o = eng.step(eng.gen_actions(40 + t, 9))
            assert all(torch.equal(x, y) for x, y in zip(o, outs[t])), t
        st = eng.get_state()
        for k in fin:
            assert np.array_equal(st[k], fin[k]), k
    c = G.TetrisBatch(n + 1, seeds=list(range(n + 1)))
    with pytest.raises(StError):
        c.load(snap)                       # other env count
    bad = bytearray(snap)
    bad[0] ^= 1
    with pytest.raises(StError):
        a.load(bytes(bad))                 # not a snapshot
    with pytest.raises(StError):
        a.load(snap[:-4])                  # truncated


@pytest.mark.parametrize("lock_delay,step_reset", [(0, False), (2, True), (3, False)])
def test_host_written_lock_fields(lock_delay, step_reset):
    """Lock-delay counters a host wrote beyond lock_delay (the reference's
    `_lock_delay_fn = (x + 1) % (max(lock_delay, 0) + 1)`, tetris_env.py:175,
    takes any x): st_step and st_rollout against the oracle with the same
    counters written into both, up to 40 with lock_mod 1, 3 and 4."""
    G = _engine()
    n, T = 512, 80
    kw = dict(width=10, height=20, lock_delay=lock_delay, step_reset=step_reset, penalise_holes_increase=True)
    seeds = [77 + e for e in range(n)]
    a = G.TetrisBatch(n, autoreset="same_step", seeds=seeds, **kw)
    b = G.TetrisBatch(n, autoreset="same_step", seeds=seeds, **kw)
    a.reset()
    b.reset()
    ob = O.OracleBatch(n, seeds, **kw)
    ob.reset()
    locks = np.random.default_rng(5).integers(0, 41, n)
    for eng in (a, b):
        p = eng.get_state(("piece",))["piece"].astype(np.int64)
        eng.set_state(piece=(p & ((1 << 17) - 1)) | (locks << 17))
    for i in range(n):
        ob.set_state(i, lock=int(locks[i]))
    acts = O.splitmix64_actions(13, 0, T, n)
    ref = ob.rollout(acts)
    ro, rr, rd = b.rollout(torch.as_tensor(acts, device=b.device))
    for t in range(T):
        o, r, d = a.step(torch.as_tensor(acts[t], device=a.device), obs="packed")
        assert np.array_equal(r.cpu().numpy(), ref["reward"][t]), t
        assert np.array_equal(d.cpu().numpy().astype(np.uint8), ref["done"][t]), t
        assert np.array_equal(o.cpu().numpy().view(np.uint32).T, ref["obs"][t]), t
        assert torch.equal(ro[t], o) and torch.equal(rr[t], r) and torch.equal(rd[t], d), t


@pytest.mark.parametrize("mode", ["step", "rollout"])
def test_host_written_large_shape_counts(mode):
    """Shape counts a host wrote far apart (st_set_state): randint's range n =
    35 + 7 max - sum reaches 2^18..2^25, so getrandbits takes 19-25 bits
    (tetris_env.py:183-191; Lib/random.py _randbelow).  The rollout's draw
    skips the tempering's last step only in waves whose lanes all draw <= 18
    bits: one wave here has none of the wide lanes, one only wide lanes, two
    a mix.  The first wave's counts spread 14..17 apart (the boundary of
    round 5's measured-and-dropped draw word).  Outputs
    and final counts / MT index vs the oracle."""
    G = _engine()
    n, T = 256, 80
    b = G.TetrisBatch(n, autoreset="same_step", seeds=range(n))
    b.reset()
    ob = O.OracleBatch(n, list(range(n)))
    ob.reset()
    st = b.get_state(("mt", "stats"))  # st_mt_sync: no preview drawn with the old counts
    mt, stats = st["mt"].copy(), st["stats"].copy()
    rng = np.random.default_rng(23)
    for i in range(n):
        if i < 64:
            counts = 50 + rng.integers(0, 18, 7)
        elif 64 <= i < 128:
            counts = np.array([100_000 + 1_000 * i, 0, 0, 0, 0, 0, 0])
        elif i >= 128 and i % 2:
            counts = rng.integers(0, 3_000_000, 7)
        else:
            counts = stats[6:13, i].astype(np.int64)
        stats[6:13, i] = counts
        e = ob.envs[i]
        for k in range(624):
            e.rng.mt[k] = int(mt[i, k])
        e.rng.index = int(stats[13, i])
        ob.set_state(i, counts=counts)
    b.set_state(mt=mt, stats=stats)
    acts = O.splitmix64_actions(9, 0, T, n)
    acts[1::2] = 2  # hard drops: a lock at least every other step
    ref = ob.rollout(acts)
    if mode == "step":
        for t in range(T):
            obs, rew, done = b.step(torch.as_tensor(acts[t], device=b.device))
            assert np.array_equal(rew.cpu().numpy(), ref["reward"][t]), t
            assert np.array_equal(obs.cpu().numpy().view(np.uint32).T, ref["obs"][t]), t
    else:
        obs, rew, done = b.rollout(torch.as_tensor(acts, device=b.device))
        assert np.array_equal(rew.cpu().numpy(), ref["reward"])
        assert np.array_equal(done.cpu().numpy().astype(np.uint8), ref["done"])
        assert np.array_equal(obs.cpu().numpy().view(np.uint32).transpose(0, 2, 1), ref["obs"])
    fin = b.get_state(("mt", "stats"))
    for i in range(n):
        assert list(fin["stats"][6:13, i].astype(np.int64)) == list(np.ctypeslib.as_array(ob.envs[i].counts)), i
        assert int(fin["stats"][13, i]) == ob.envs[i].rng.index, i


def test_step_n_equals_k_step_calls():
    """st_step_n (ABI 4, the bench's native launch loop): k steps enqueued by
    one call -- step i with the actions at d_actions[i] -- leave the same
    state and last-step outputs as k st_step calls, packed and float32;
    k = 0 enqueues nothing."""
    import ctypes
    G = _engine()
    n, k = 3000, 37
    for f32 in (False, True):
        a = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=False)
        b = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=False)
        a.reset()
        b.reset()
        acts = torch.stack([b.gen_actions(t, 11) for t in range(k)])
        vp = ctypes.c_void_p
        arr = (vp * k)(*[acts[t].data_ptr() for t in range(k)])
        o = torch.zeros((10, n), dtype=torch.int32, device=a.device)
        r = torch.zeros(n, dtype=torch.int32, device=a.device)
        d = torch.zeros(n, dtype=torch.uint8, device=a.device)
        f = torch.zeros((n, 10, 20), dtype=torch.float32, device=a.device) if f32 else None
        s = vp(torch.cuda.current_stream().cuda_stream)
        assert a._L.st_step_n(a._ctx, vp(ctypes.addressof(arr)), 0, vp(o.data_ptr()), None, vp(r.data_ptr()),
                              vp(d.data_ptr()), s) == 0
        assert a._L.st_step_n(a._ctx, vp(ctypes.addressof(arr)), k, vp(o.data_ptr()),
                              vp(f.data_ptr()) if f32 else None, vp(r.data_ptr()), vp(d.data_ptr()), s) == 0
        for t in range(k):
            ob, rb, db = b.step(acts[t], obs="f32" if f32 else "packed")
        torch.cuda.synchronize()
        if f32:
            assert torch.equal(f, ob)
            ob = b.obs
        assert torch.equal(o, ob) and torch.equal(r, rb) and torch.equal(d.bool(), db.bool())
        sa, sb = a.get_state(("board", "stats", "mt")), b.get_state(("board", "stats", "mt"))
        for key in sa:
            assert np.array_equal(sa[key], sb[key]), (key, f32)
        a.close()
        b.close()


@pytest.mark.parametrize("obs", ["packed", "f32", "none"])
def test_engine_step_n_equals_step_calls(obs):
    """TetrisBatch.step_n (st_step_n behind it): K rows of actions, the last
    step's outputs and every env's state as K step() calls; a bad action
    raises KeyError before any step with validate_actions=True."""
    G = _engine()
    n, k = 1500, 23
    a = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=True)
    b = G.TetrisBatch(n, seeds=range(n), autoreset="same_step", validate_actions=False)
    a.reset()
    b.reset()
    acts = torch.stack([b.gen_actions(t, 5) for t in range(k)])
    oa, ra, da = a.step_n(acts, obs=obs)
    for t in range(k):
        ob, rb, db = b.step(acts[t], obs=obs)
    torch.cuda.synchronize()
    assert (oa is None) == (ob is None) and (oa is None or torch.equal(oa, ob))
    assert torch.equal(ra, rb) and torch.equal(da, db)
    sa, sb = a.get_state(("board", "stats", "mt")), b.get_state(("board", "stats", "mt"))
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    bad = acts.clone()
    bad[3, 7] = 9
    before = a.get_state(("board", "stats", "mt"))
    before = {key: v.copy() for key, v in before.items()}
    with pytest.raises(KeyError):
        a.step_n(bad, obs=obs)
    after = a.get_state(("board", "stats", "mt"))
    for key in before:
        assert np.array_equal(before[key], after[key]), key
    a.close()
    b.close()
