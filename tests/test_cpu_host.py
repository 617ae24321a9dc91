"""CPU-only tests: the C-ABI library loads and exports every symbol the public
header declares (no compute calls), host-side logic (sharding, gather packing
over gloo with world_size 2, spaces, make), and that the product path refuses
to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from replay import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "simpletetris.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(st_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from gym_simpletetris_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = header_functions()
    assert len(names) >= 12
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(_lib.EXPORTS)


def test_host_only_abi_functions_and_constants():
    """The C ABI's pure host functions (no GPU call) and the header constants
    the Python binding mirrors."""
    from gym_simpletetris_amd import _lib
    L = _lib.load()
    assert L.st_abi_version() == _lib.ABI_VERSION == 4
    assert L.st_export_words(10, 20) == 10 + 2 + _lib.NSTAT + _lib.MT_N + 200
    assert L.st_export_words(4, 4) == 4 + 2 + _lib.NSTAT + _lib.MT_N + 16
    # the C5 gather format: ceil((W*H + 17) / 32) words per env
    assert L.st_wire_words(10, 20) == 8 and L.st_wire_words(32, 28) == 30 and L.st_wire_words(4, 4) == 2
    assert L.st_wire_words(0, 20) == _lib.ST_EINVAL and L.st_wire_words(10, 29) == _lib.ST_EINVAL
    assert L.st_unwire(10, 20, -1, None, None, None, None, None) == _lib.ST_EINVAL
    src = open(os.path.join(ROOT, "include", "simpletetris.h")).read()
    defs = dict(re.findall(r"#define\s+(ST_EXPORT_\w+)\s+(\d+)u", src))
    assert int(defs["ST_EXPORT_MT"]) == _lib.EXPORT_MT and int(defs["ST_EXPORT_OBS_F32"]) == _lib.EXPORT_OBS_F32
    assert int(re.search(r"\bST_NSTAT\s*=\s*(\d+)", src).group(1)) == _lib.NSTAT  # enum constant
    assert int(re.search(r"#define\s+ST_ABI_VERSION\s+(\d+)", src).group(1)) == _lib.ABI_VERSION
    # argument checks that return before any GPU call
    assert L.st_gate_actions(None, None, None) == _lib.ST_EINVAL
    assert L.st_gate_wait(None) == _lib.ST_EINVAL
    assert L.st_step_n(None, None, 3, None, None, None, None, None) == _lib.ST_EINVAL
    assert L.st_stream_wait(None, None) == _lib.ST_OK  # a stream never waits for itself


def test_abi_mismatch_refused_unless_old_abi_opt_in(tmp_path, monkeypatch):
    """A library of another ABI version is refused even when ST_LIB points at
    it; only ST_AB_OLD_ABI=1 (diagnostic A/Bs) loads it, with a warning
    (ADVICE r5)."""
    import importlib
    import subprocess
    import sys
    src = tmp_path / "old.c"
    src.write_text("int st_abi_version(void) { return 1; }\n")
    so = tmp_path / "libold.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    code = ("import sys; sys.path.insert(0, %r); from gym_simpletetris_amd import _lib\n"
            "try:\n    _lib.load()\nexcept ImportError as e:\n    print('refused', e)\nelse:\n    print('loaded')")
    pkg = os.path.join(ROOT, "gym-simpletetris_amd")
    env = dict(os.environ, ST_LIB=str(so))
    env.pop("ST_AB_OLD_ABI", None)
    out = subprocess.run([sys.executable, "-c", code % pkg], env=env, capture_output=True, text=True)
    assert out.stdout.startswith("refused") and "ABI 1" in out.stdout, out.stdout + out.stderr
    env["ST_AB_OLD_ABI"] = "1"
    out = subprocess.run([sys.executable, "-W", "always", "-c", code % pkg], env=env, capture_output=True, text=True)
    assert out.stdout.startswith("loaded") and "ST_AB_OLD_ABI" in out.stderr, out.stdout + out.stderr


def test_library_is_gfx950_code_object():
    from gym_simpletetris_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"k_step" in data


def test_no_cpu_fallback():
    import gym_simpletetris_amd as G
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="GPU"):
        G.TetrisBatch(4)


def test_make_ids():
    import gym_simpletetris_amd as G
    with pytest.raises(KeyError):
        G.make("SimpleTetris-v1")


def test_scalar_action_follows_the_reference_dict():
    """value_action_map[a] (tetris_env.py:152-160, :245): the keys are the
    ints 0..6; equal numbers of other types hit them (True, 2.0, np.int8),
    anything else raises KeyError."""
    from gym_simpletetris_amd.engine import scalar_action
    ref = {i: i for i in range(7)}
    for a in (0, 6, 2.0, np.float32(5.0), np.int64(3), np.uint8(1), True, False):
        assert scalar_action(a) == ref[a]
    for a in (7, -1, 2.5, float("nan"), float("inf"), "2", None, np.float64(6.5)):
        with pytest.raises(KeyError):
            scalar_action(a)
        with pytest.raises((KeyError, TypeError)):
            ref[a]


def test_import_leaves_hip_environment_alone():
    """Importing the package changes no process-wide HIP setting;
    tune_runtime() is the explicit opt-in."""
    import subprocess
    import sys
    code = ("import os, sys; sys.path.insert(0, 'gym-simpletetris_amd'); "
            "os.environ.pop('HIP_FORCE_DEV_KERNARG', None); import gym_simpletetris_amd as G; "
            "assert 'HIP_FORCE_DEV_KERNARG' not in os.environ; "
            "assert G.tune_runtime() and os.environ['HIP_FORCE_DEV_KERNARG'] == '1'; print('ok')")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr[-2000:]


def test_spaces_stand_ins():
    from gym_simpletetris_amd import spaces
    d = spaces.Discrete(7)
    assert d.n == 7 and d.contains(3) and not d.contains(7)
    b = spaces.Box(0, 1, shape=(10, 20), dtype=np.float32)
    assert b.shape == (10, 20) and b.dtype == np.float32


def test_shard_range_covers_exactly():
    from gym_simpletetris_amd.distributed import shard_range
    for n in (1, 7, 64, 65536 * 8, 1000003):
        for world in (1, 2, 3, 4, 8):
            if world > n:
                continue
            seen = 0
            for r in range(world):
                off, cnt = shard_range(n, world, r)
                assert off == seen
                seen += cnt
            assert seen == n


def test_grayscale_closed_form_matches_reference_images():
    """The per-pixel formula st_grayscale evaluates (R19), restated in numpy,
    equals convert_grayscale's output recorded from the reference."""
    d = np.load(os.path.join(GOLDEN, "grayscale.npz"))
    for i, (W, H) in enumerate(d["dims"]):
        board = d["boards"][i][:W, :H]
        for size, key in ((84, "g84"), (160, "g160")):
            lim = max(W, H)
            gap = size // 100 + 1
            blk = (size - 2 * gap) // lim - gap
            pitch = blk + gap
            pr = (size - (gap + pitch * H)) // 2
            pc = (size - (gap + pitch * W)) // 2
            r = np.arange(size)[:, None] - pr
            c = np.arange(size)[None, :] - pc
            inside = (r >= 0) & (c >= 0) & (r < gap + pitch * H) & (c < gap + pitch * W)
            cell = inside & (r % pitch >= gap) & (c % pitch >= gap)
            y = np.clip(r // pitch, 0, H - 1)
            x = np.clip(c // pitch, 0, W - 1)
            img = np.where(inside, 128, 0)
            img = np.where(cell & (board[x, y] != 0), 190, img)
            assert np.array_equal(img, d[key][i]), (i, size)


def _gather_worker(rank, world, port, q, n_global):
    import torch.distributed as dist
    from gym_simpletetris_amd.distributed import (assemble, buffer_views, gather_outputs,
                                                  output_buffer, shard_cap, shard_range)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W = 10
    off, n = shard_range(n_global, world, rank)
    buf = output_buffer(W, n, "cpu")
    obs, rew, done = buffer_views(buf, W)
    g = torch.arange(off, off + n, dtype=torch.int32)
    obs[:] = g[None, :] * 16 + torch.arange(W, dtype=torch.int32)[:, None]
    rew[:] = -g
    done[:] = (g % 3 == 0).to(torch.uint8)
    bufs = gather_outputs(buf, n_cap=shard_cap(n_global, world))
    if rank == 0:
        o, r, d = assemble(bufs, W, [shard_range(n_global, world, i)[1] for i in range(world)])
        ok = (torch.equal(r, -torch.arange(n_global, dtype=torch.int32))
              and d.dtype == torch.bool and torch.equal(d, torch.arange(n_global) % 3 == 0)
              and torch.equal(o[3], torch.arange(n_global, dtype=torch.int32) * 16 + 3))
        q.put(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_global", [(2, 64), (2, 67), (3, 67)])
def test_gather_packing_gloo(world, n_global):
    """Even and ragged shards (short ranks send a padded buffer)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q, n_global))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def test_algorithmic_bytes_formula():
    import bench
    b = bench.algorithmic_bytes(10, 20, 0.0, False)
    assert b == (1 + 4 + 4 + 40) + (4 + 4 + 4 + 1 + 40)
    assert bench.algorithmic_bytes(10, 20, 0.0, True) == b + 800
    assert bench.algorithmic_bytes(10, 20, 1.0, False) > b


def test_bench_roofline_bytes_and_pmc_tie(tmp_path, monkeypatch):
    """bench.py prices a launch with PMC traffic / rocprof durations only
    from a summary of the same kernel sources AND the same launch shape
    (kernel, grid, steps per launch); the summary tools key them so."""
    import json
    import sys
    import bench
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_summary
    assert bench.s8d_bytes(0.0, False) == 182 and bench.s8d_bytes(1.0, False) == 366
    assert bench.s8d_bytes(0.5, True) == 902 + 92
    assert abs(bench.algorithmic_bytes(10, 20, 1.0, False) - (102 + 167.7)) < 1e-9
    assert bench.step_grid(4096) == 8192 and bench.step_grid(65536) == 131072
    assert len(bench.kernel_source_sha()) == 16
    step = bench.launch_key("k_step<10, 20, false, false, true, false>", bench.step_grid(65536), 1)
    ro = bench.launch_key("k_rollout<10, 20, false, true>", bench.step_grid(65536), 100)
    assert step.endswith("@131072@k1") and ro.endswith("@131072@k100")
    assert pmc_summary.launch_k("void st::(anonymous namespace)::k_rollout<10, 20, false, true>(st::KParams)", 100) == 100
    assert pmc_summary.launch_k("void st::(anonymous namespace)::k_step<10, 20, false, false, true, false>(st::KParams)", 100) == 1
    sha = bench.kernel_source_sha()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "rX_pmc.json").write_text(json.dumps({"kernel_source_sha": sha, "kernels": {
        step: {"hbm_bytes_per_launch": 1.5e7}, ro: {"hbm_bytes_per_launch": 3e8}}}))
    (prof / "rX_trace.json").write_text(json.dumps({"kernel_source_sha": sha, "kernels": {
        step: {"mean_us": 5.0, "median_us": 4.9, "launches": 4000, "trace": "t.csv", "p_lock": 0.2}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got, src = bench.load_pmc(step, sha)
    assert got == 1.5e7 and src == "rX_pmc.json"
    assert bench.load_pmc(ro, sha)[0] == 3e8
    # another launch shape (a 20-step rollout) or other sources: no number
    got, why = bench.load_pmc(ro.replace("@k100", "@k20"), sha)
    assert got is None and "launch shape" in why
    assert bench.load_pmc(step, "0" * 16)[0] is None
    tr = bench.load_trace(step, sha)
    assert tr["launches"] == 4000 and tr["p_lock"] == 0.2 and tr["source"] == "rX_trace.json"
    assert bench.load_trace(step, "0" * 16) is None
    # p_lock per launch key from a bench JSON line's roofline objects
    bj = tmp_path / "b.json"
    bj.write_text("noise\n" + json.dumps({"roofline": {"launch_key": step, "p_lock": 0.21},
                                          "variants": {"rollout_packed": {"roofline": {"launch_key": ro, "p_lock": 0.2}},
                                                       "note": "x"}}))
    assert pmc_summary.bench_p_lock(str(bj)) == {step: 0.21, ro: 0.2}
    # the image kernels' launch keys as bench.py derives them
    for ch in (1, 3):
        name, grid = bench.image_launch(65536, 84, ch, False)
        assert name.startswith("k_grayscale") and grid > 0


def test_committed_profiles_match_sources():
    """The newest committed PMC and trace summaries describe the committed
    kernel sources (so the bench line's traffic / rocprof are not null) and
    carry launch-shape keys."""
    import glob
    import json
    import bench
    pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    trs = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_trace.json")))
    d, tj = json.load(open(pmcs[-1])), json.load(open(trs[-1]))
    assert d["kernel_source_sha"] == tj["kernel_source_sha"] == bench.kernel_source_sha()
    head = bench.launch_key("k_step<10, 20, false, false, true, false>", bench.step_grid(65536), 1)
    assert head in d["kernels"] and head in tj["kernels"]
    assert tj["kernels"][head]["p_lock"] is not None


def test_bench_cpu_baseline_all_cores():
    import bench
    cb = bench.cpu_baseline(0.2, "c4")
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0 and cb["single_core"] > 0
    assert cb["nproc"] >= 1 and cb["cpu_model"]


def test_dlpack_producer_passes_through_without_copy():
    from gym_simpletetris_amd.engine import _from_dlpack

    class Foreign:
        def __init__(self, t):
            self.t = t

        def __dlpack__(self, stream=None, **kw):
            return self.t.__dlpack__()

        def __dlpack_device__(self):
            return self.t.__dlpack_device__()
    t = torch.arange(7, dtype=torch.uint8)
    u = _from_dlpack(Foreign(t))
    assert isinstance(u, torch.Tensor) and u.data_ptr() == t.data_ptr() and torch.equal(u, t)
    assert _from_dlpack(t) is t
    a = np.arange(3)
    assert _from_dlpack(a) is a


def test_bench_distinct_devices_counts_physical_gpus():
    """bench.py --gpus N refuses to run when fewer distinct GPUs than ranks
    answer; the count must not mistake distinct GPUs for one when a field is
    degenerate (all-zero UUIDs), nor one shared GPU for several."""
    import bench

    def ident(uuid, bus, host="h"):
        d = {"host": host, "pci_domain_id": "0", "pci_bus_id": bus, "pci_device_id": "0"}
        if uuid is not None:
            d["uuid"] = uuid
        d["device_key"] = "uuid:%s" % uuid if uuid else "pci:%s" % bus
        return d
    shared = [ident("35383437-6461", "139")] * 8
    assert bench.distinct_devices(shared) == 1
    distinct = [ident("u%d" % i, str(100 + i)) for i in range(8)]
    assert bench.distinct_devices(distinct) == 8
    zero_uuid = [ident("00000000-0000-0000-0000-000000000000", str(100 + i)) for i in range(8)]
    assert bench.distinct_devices(zero_uuid) == 8
    same_uuid_distinct_pci = [ident("35383437", str(100 + i)) for i in range(4)]
    assert bench.distinct_devices(same_uuid_distinct_pci) == 4
    no_fields = [{"host": "h", "device_key": "idx:h:None:%d" % i} for i in range(2)]
    assert bench.distinct_devices(no_fields) == 2
