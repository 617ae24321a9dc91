"""The N > 1 path on one GPU box (VERDICT r1 "next" #2).

1. Two rank processes (torch.distributed, gloo: both ranks share cuda:0 on a
   one-GPU box) each step their ShardedTetris shard of a (2n + 1)-env batch
   (ragged: rank 0 holds one env more, so rank 1 sends a padded buffer) and
   gather the packed obs / reward / done to rank 0 every step; rank 0's
   assembled global outputs must equal one process stepping all 2n + 1 envs
   (the split is by global env index: seeds and actions keyed by it).
2. `python bench.py --gpus 2` run directly (no torch.distributed.run): it
   starts its own two ranks and prints one JSON line with the gather variant.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_LOCAL, T, SEED, ASEED = 3000, 150, 500, 0x77

WORKER = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [{root!r}, os.path.join({root!r}, "gym-simpletetris_amd")]
from gym_simpletetris_amd.distributed import ShardedTetris
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
sh = ShardedTetris({n_global}, seed={seed}, device=torch.device("cuda", 0), autoreset="same_step",
                   penalise_holes_increase=True)
sh.reset()
obs, rew, done = [], [], []
for t in range({steps}):
    a = sh.engine.gen_actions(t, {aseed}, global_offset=sh.offset).clone()
    sh.step(a)
    torch.cuda.synchronize()
    bufs = sh.gather(cpu=True)
    if rank == 0:
        o, r, d = sh.assemble(bufs)
        obs.append(o.numpy()); rew.append(r.numpy()); done.append(d.numpy())
if rank == 0:
    np.savez({out!r}, obs=np.stack(obs), rew=np.stack(rew), done=np.stack(done))
dist.barrier()
dist.destroy_process_group()
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_gather_equals_one_batch(tmp_path):
    out = str(tmp_path / "gathered.npz")
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, n_global=2 * N_LOCAL + 1, seed=SEED, steps=T, aseed=ASEED,
                                    out=out))
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env))
    rcs = [p.wait(timeout=100) for p in procs]
    assert rcs == [0, 0]
    got = np.load(out)

    import gym_simpletetris_amd as G
    n = 2 * N_LOCAL + 1
    b = G.TetrisBatch(n, autoreset="same_step", seeds=[SEED + e for e in range(n)],
                      penalise_holes_increase=True)
    b.reset()
    for t in range(T):
        o, r, d = b.step(b.gen_actions(t, ASEED))
        assert np.array_equal(r.cpu().numpy(), got["rew"][t]), t
        assert np.array_equal(d.cpu().numpy().astype(np.uint8), got["done"][t]), t
        assert np.array_equal(o.cpu().numpy(), got["obs"][t]), t
    assert got["done"].any()  # auto-resets happened inside the compared span


def check_bench_dump(path, n_global, steps):
    """bench.py's C5 region (ST_BENCH_DUMP): rank 0's assembled outputs of the
    last timed step -- gathered from every rank -- against the oracle stepping
    all n_global envs through the same `steps` action rows (seeds 1000 + e,
    the bench's splitmix64 actions keyed by the global index)."""
    from test_gpu_long_horizon import ParallelOracle
    z = np.load(path)
    assert int(z["n_global"]) == n_global and int(z["step"]) == steps - 1
    orc = ParallelOracle(n_global, {})
    try:
        if steps > 1:
            orc.rollout(0, steps - 1, obs=False)
        ref = orc.rollout(steps - 1, 1)
    finally:
        orc.close()
    assert np.array_equal(z["reward"], ref["reward"][0])
    assert np.array_equal(z["done"].astype(np.uint8), ref["done"][0])
    assert np.array_equal(z["obs"].T, ref["obs"][0])
    return z


def test_bench_gpus2_direct_invocation(tmp_path):
    """bench.py --gpus 2 with the row gather format (st_step's obs / reward /
    done rows; the 8-rank test covers the default wire format)."""
    env = dict(os.environ, ST_BENCH_SHARED_GPU="1", ST_BENCH_DUMP=str(tmp_path / "c5.npz"))
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "30", "--warmup", "5", "--n-envs", "8192", "--no-cpu-baseline",
                        "--no-clear-heavy", "--gather-format", "rows"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["envs_total"] == 2 * 8192
    # both ranks reported in; they share cuda:0 here (ST_BENCH_SHARED_GPU)
    assert d["ranks_seen"] == 2 and d["distinct_devices"] == 1 and d["rccl_version"] is None
    assert d["value"] > 0 and d["gather"]["gathers_in_timed_region"] == 30
    assert d["gather"]["bytes_per_rank_per_step"] == (10 + 2) * 8192 * 4
    assert d["step_no_gather"]["value"] > 0
    assert d["scaling"] == "weak"
    z = check_bench_dump(tmp_path / "c5.npz", 2 * 8192, 35)
    assert int(z["gathers_timed"]) == 30


def test_bench_rccl_calls_one_rank(tmp_path):
    """The nccl (RCCL) side of bench.py on a one-GPU box: init with device_id,
    barriers, the MAX all-reduce of the timings and the double-buffered async
    gather of the C5 region, at one rank (two ranks cannot share a GPU under
    RCCL); the gathered outputs of the last timed step equal the oracle's."""
    env = dict(os.environ, ST_BENCH_FORCE_DIST="1", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), ST_BENCH_DUMP=str(tmp_path / "c5.npz"))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--backend", "nccl",
                        "--steps", "30", "--warmup", "5", "--n-envs", "8192", "--no-cpu-baseline",
                        "--no-clear-heavy"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["gather"]["backend"] == "nccl" and d["gather"]["gathers_in_timed_region"] == 30
    assert d["gather"]["decodes_in_timed_region_rank0"] == 30  # wire format: decoded inside the region
    assert d["value"] > 0
    # the self-verifying topology keys the driver's N-GPU record carries
    assert d["ranks_seen"] == 1 and d["distinct_devices"] == 1
    assert d["rccl_version"] and not str(d["rccl_version"]).startswith("unknown")
    assert d["topology"]["backend"] == "nccl" and d["topology"]["devices"][0]["rank"] == 0
    z = check_bench_dump(tmp_path / "c5.npz", 8192, 35)
    assert int(z["decodes_timed"]) == 30
