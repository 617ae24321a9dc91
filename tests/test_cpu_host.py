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
    assert L.st_abi_version() == 1
    assert L.st_export_words(10, 20) == 10 + 2 + _lib.NSTAT + _lib.MT_N + 200
    assert L.st_export_words(4, 4) == 4 + 2 + _lib.NSTAT + _lib.MT_N + 16
    src = open(os.path.join(ROOT, "include", "simpletetris.h")).read()
    defs = dict(re.findall(r"#define\s+(ST_EXPORT_\w+)\s+(\d+)u", src))
    assert int(defs["ST_EXPORT_MT"]) == _lib.EXPORT_MT and int(defs["ST_EXPORT_OBS_F32"]) == _lib.EXPORT_OBS_F32
    assert int(re.search(r"\bST_NSTAT\s*=\s*(\d+)", src).group(1)) == _lib.NSTAT  # enum constant


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
              and torch.equal(d, (torch.arange(n_global) % 3 == 0).to(torch.uint8))
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


def test_bench_roofline_bytes_and_pmc_tie():
    import json
    import bench
    assert bench.s8d_bytes(0.0, False) == 182 and bench.s8d_bytes(1.0, False) == 366
    assert bench.s8d_bytes(0.5, True) == 902 + 92
    assert abs(bench.algorithmic_bytes(10, 20, 1.0, False) - (102 + 167.7)) < 1e-9
    # traffic is taken only from a PMC summary of the same kernel sources
    pmc = os.path.join(ROOT, "profiles", "r02_pmc.json")
    d = json.load(open(pmc))
    kname = "k_step<10, 20, false, false, true>@%d" % bench.step_grid(65536)
    got, src = bench.load_pmc(kname, d["kernel_source_sha"])
    assert src == "r02_pmc.json" and got == d["kernels"][kname]["hbm_bytes_per_launch"]
    assert bench.step_grid(4096) == 8192 and bench.step_grid(65536) == 131072
    got, why = bench.load_pmc(kname, "0" * 16)
    assert got is None and "no PMC pass" in why
    assert len(bench.kernel_source_sha()) == 16
    # the rocprofv3 trace stats come the same way, from a trace of the same sources
    tj = json.load(open(os.path.join(ROOT, "profiles", "r02_trace.json")))
    tr = bench.load_trace(kname, tj["kernel_source_sha"])
    assert tr["launches"] == tj["kernels"][kname]["launches"] and tr["source"] == "r02_trace.json"
    assert bench.load_trace(kname, "0" * 16) is None
    # the image kernels' launch keys as bench.py derives them are the ones the
    # PMC pass recorded (launch_grayscale's choice of kernel and grid)
    for ch in (1, 3):
        key = "%s@%d" % bench.image_launch(65536, 84, ch, False)
        assert key in d["kernels"], key
    # the committed profiles describe the committed kernel sources
    assert d["kernel_source_sha"] == tj["kernel_source_sha"] == bench.kernel_source_sha()


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
