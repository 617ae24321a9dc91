"""BASELINE config C5 at its own shape, on one GPU box (VERDICT r2 "next" #1).

C5 is 524,288 10x20 boards sharded over 8 GPUs, every shard's packed obs /
reward / done gathered to rank 0.  The pool gives one GPU per box, so the 8
ranks here are 8 processes on cuda:0 talking gloo (RCCL needs one GPU per
rank); everything else is the C5 path: `ShardedTetris(524_288)` per rank
(contiguous global-index shards, seeds 1000 + e, the bench's splitmix64
actions keyed by the global index, same-step auto-reset), a gather to rank 0
after EVERY step, and `assemble()` on rank 0.  Rank 0 checks the assembled
global outputs of every step, and then every shard's final state (board,
piece, counters, MT19937 index and words), bit-exact against the oracle
stepping all 524,288 envs -- the reference has no shared state but its global
`random` (tetris_env.py:187), which the engine replaces by per-env streams,
so the result must not depend on the rank count.  A ragged case (8 x 4,096
+ 3 envs: rank 0..2 hold one env more, the others send zero-padded buffers)
runs the padding path of `gather_outputs` / `assemble`.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 8

WORKER = r"""
import os, sys, time
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [{root!r}, os.path.join({root!r}, "gym-simpletetris_amd"), os.path.join({root!r}, "tests")]
from gym_simpletetris_amd.distributed import ShardedTetris, shard_range
NG, T, CH, W, H = {n_global}, {steps}, {chunk}, 10, 20
SEED, ASEED = 1000, 0x5EED
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
sh = ShardedTetris(NG, seed=SEED, device=dev, autoreset="same_step", width=W, height=H)
assert sh.n == shard_range(NG, world, rank)[1]
sh.reset()
acts = torch.empty(sh.n, dtype=torch.uint8, device=dev)
orc = None
if rank == 0:
    from test_gpu_long_horizon import ParallelOracle, _pack_board
    orc = ParallelOracle(NG, {{}})
t_start = time.time()
deaths = 0
for t0 in range(0, T, CH):
    got = []
    for t in range(t0, t0 + CH):
        sh.engine.gen_actions(t, ASEED, global_offset=sh.offset, out=acts)
        sh.step(acts)
        bufs = sh.gather(cpu=True)  # every step, to rank 0
        if rank == 0:
            o, r, d = sh.assemble(bufs)
            assert o.shape == (W, NG) and r.shape == (NG,) and d.shape == (NG,)
            got.append((o.numpy().view(np.uint32).copy(), r.numpy().copy(), d.numpy().copy()))
    if rank == 0:
        ref = orc.rollout(t0, CH)
        for i, (o, r, d) in enumerate(got):
            assert np.array_equal(r, ref["reward"][i]), ("reward", t0 + i)
            assert np.array_equal(d.astype(np.uint8), ref["done"][i]), ("done", t0 + i)
            bad = np.argwhere(o.T != ref["obs"][i])
            assert bad.size == 0, ("obs", t0 + i, bad[:4])
            deaths += int(d.sum())
        print("rank 0: steps %d..%d bit-exact (%.0f s)" % (t0, t0 + CH - 1, time.time() - t_start), flush=True)
# final state of every shard, gathered to rank 0 (padded to the largest shard)
st = sh.engine.get_state()  # st_mt_sync first: CPython's MT state
mt = st["mt"].astype(np.uint64)
mult = (2 * np.arange(mt.shape[1], dtype=np.uint64) + 1)[None, :]
with np.errstate(over="ignore"):
    fold = (mt * mult).sum(axis=1, dtype=np.uint64)  # mod 2^64
rows = np.concatenate([st["board"].astype(np.int64), st["stats"].astype(np.int64),
                       st["piece"].astype(np.int64)[None, :], fold.view(np.int64)[None, :]])
send = torch.zeros((rows.shape[0], sh.n_cap), dtype=torch.int64)
send[:, :sh.n] = torch.from_numpy(rows)
gl = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
dist.gather(send, gather_list=gl, dst=0)
if rank == 0:
    fin = np.concatenate([g.numpy()[:, :c] for g, c in zip(gl, sh.counts)], axis=1)
    ref = orc.final_state()
    brd, stats, piece, fold = fin[:W], fin[W:W + 19], fin[W + 19].astype(np.uint32), fin[W + 20].view(np.uint64)
    assert np.array_equal(brd.astype(np.uint32), _pack_board(ref["board"])), "board"
    for row, field in ((0, "time"), (1, "score"), (2, "lines_cleared"), (3, "holes"),
                       (4, "piece_height"), (5, "n_deaths")):
        assert np.array_equal(stats[row], ref[field]), field
    assert np.array_equal(stats[6:13].T, ref["counts"]), "shape counts"
    for name, v in (("shape_id", piece & 7), ("rot", (piece >> 3) & 3), ("ax", (piece >> 5) & 63),
                    ("ay", (piece >> 11) & 63), ("lock", piece >> 17)):
        assert np.array_equal(v.astype(np.int64), ref[name].astype(np.int64)), name
    assert np.array_equal(stats[13], ref["rng"]["index"]), "MT index"
    rmt = ref["rng"]["mt"].astype(np.uint64)
    with np.errstate(over="ignore"):
        rfold = (rmt * mult).sum(axis=1, dtype=np.uint64)
    assert np.array_equal(fold, rfold), "MT words"
    assert deaths > NG // 4  # auto-resets happened inside the compared span
    orc.close()
    print("C5 OK", flush=True)
dist.barrier()
dist.destroy_process_group()
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, n_global, steps, chunk, timeout):
    script = tmp_path / "c5_worker.py"
    script.write_text(WORKER.format(root=ROOT, n_global=n_global, steps=steps, chunk=chunk))
    port = _port()
    procs = []
    logs = []
    # rank logs under gpurun_out/ when it exists (a long run then shows progress there)
    logdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else str(tmp_path)
    tag = f"c5_{n_global}"
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="1")
        log = open(os.path.join(logdir, f"{tag}_rank{r}.log"), "w")
        logs.append(log)
        procs.append(subprocess.Popen([sys.executable, "-u", str(script)], env=env, stdout=log,
                                      stderr=subprocess.STDOUT))
    try:
        rcs = [p.wait(timeout=timeout) for p in procs]
    finally:
        for p in procs:  # a failed rank leaves the others in a collective
            if p.poll() is None:
                p.kill()
                p.wait()
        for log in logs:
            log.close()
    out0 = open(os.path.join(logdir, f"{tag}_rank0.log")).read()
    errs = "".join(open(os.path.join(logdir, f"{tag}_rank{r}.log")).read()[-1500:]
                   for r in range(WORLD) if rcs[r] != 0)
    assert rcs == [0] * WORLD, errs or out0[-3000:]
    assert "C5 OK" in out0, out0[-3000:]
    return out0


@pytest.mark.timeout(600)
def test_c5_eight_ranks_full_shape(tmp_path):
    """524,288 envs = 8 x 65,536, 200 steps, gathered every step."""
    out = _run_ranks(tmp_path, 8 * 65536, 200, 10, timeout=600)
    print(out[-400:])


@pytest.mark.timeout(400)
def test_c5_eight_ranks_ragged(tmp_path):
    """8 x 4,096 + 3 envs (ranks 0-2 one env more; the others send padded
    buffers), 300 steps."""
    _run_ranks(tmp_path, 8 * 4096 + 3, 300, 50, timeout=300)


@pytest.mark.timeout(400)
def test_bench_gpus8_direct_invocation(tmp_path):
    """`python bench.py --gpus 8` run directly: it spawns its 8 ranks itself
    (the driver's C5 launch path, here all on cuda:0 over gloo); every timed
    step is st_step_wire on each shard + the gather to rank 0 + rank 0's
    decode of the gathered rows (K gathers and K decodes inside the region),
    and rank 0's decoded outputs of the last timed step equal the oracle
    stepping all 8 x 2,048 envs.  Rank 0 prints one JSON line."""
    from test_gpu_multirank import check_bench_dump
    dump = tmp_path / "c5.npz"
    env = dict(os.environ, ST_BENCH_SHARED_GPU="1", ST_BENCH_DUMP=str(dump))
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--backend", "gloo",
                        "--steps", "20", "--warmup", "5", "--n-envs", "2048", "--no-cpu-baseline",
                        "--no-clear-heavy", "--no-surfaces"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["envs_total"] == 8 * 2048
    # every rank's device identity arrived over the process group; all eight
    # share cuda:0 on this box (ST_BENCH_SHARED_GPU), so one distinct device
    assert d["ranks_seen"] == 8 and d["distinct_devices"] == 1
    assert sorted(x["rank"] for x in d["topology"]["devices"]) == list(range(8))
    assert d["value"] > 0 and d["gather"]["gathers_in_timed_region"] == 20
    # the default gather format: st_step_wire's 8 rows per env, not W + 2
    assert d["gather"]["bytes_per_rank_per_step"] == 8 * 2048 * 4
    # rank 0 decoded every timed step's gathered rows inside the region
    assert d["gather"]["decodes_in_timed_region_rank0"] == 20
    assert d["gather"]["no_decode"]["value"] > 0
    assert d["gather"]["format"].startswith("st_step_wire")
    assert d["config"]["workload"].startswith("C5:")
    assert d["scaling"] == "weak"
    z = check_bench_dump(dump, 8 * 2048, 25)  # the region's own last decode vs the oracle
    assert int(z["gathers_timed"]) == 20 and int(z["decodes_timed"]) == 20
