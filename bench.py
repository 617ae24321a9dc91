#!/usr/bin/env python
"""bench.py -- env-steps/s of the MI355X batched SimpleTetris engine.

Metric (BASELINE.json): env-steps/sec at 65,536 parallel 10x20 boards per GPU,
1 -> 8 GPU weak scaling.  One "step" = one batched TetrisEngine.step
(tetris_env.py:243-304) over every env of the job (one st_step launch per
GPU), fed by synthetic uniform actions a[t, e] = splitmix64(seed ^ ((t << 32)
^ e)) % 7 that are generated into HBM before the timed region.
Envs auto-reset inside the step kernel when they die (the reference driver's
`if done: env.reset()`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4] [--obs packed|f32]

--gpus N > 1: one process per GPU.  Run directly, bench.py starts the N rank
processes itself (before anything touches a GPU) with the rendezvous on
127.0.0.1; under torch.distributed.run it is one of the ranks.  Each rank owns
a contiguous block of global env indices (seeds and actions keyed by the
global index, so the work is identical at any N; "scaling": "weak"), and each
timed step is BASELINE config C5's step: st_step_wire on every shard, the
RCCL gather of every shard's packed obs/reward/done to rank 0, double-buffered
(step t+1 computes into the other buffer while the gather of step t runs), and
rank 0's decode of the gathered rows into the global obs / reward / done
(st_unwire_shards).  The same steps without the decode (`gather.no_decode`)
and without the gather (`step_no_gather`) are reported beside it.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
sys.path.insert(0, ROOT)
# Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1): the package's
# documented opt-in (gym_simpletetris_amd.tune_runtime(); importing it sets
# nothing), which bench.py takes before the HIP runtime starts, as a
# step-per-launch user would (profiles/r02_ab_env.txt).  An
# explicit setting in the environment wins; the line records which applied.
KERNARG_FROM_ENV = bool(os.environ.get("HIP_FORCE_DEV_KERNARG"))
if not KERNARG_FROM_ENV:
    os.environ["HIP_FORCE_DEV_KERNARG"] = "1"

import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
try:
    METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
except Exception:  # noqa: BLE001
    METRIC = "env-steps/sec at 65 536 parallel 10×20 boards; 1→8 GPU scaling"

CONFIGS = {
    # BASELINE.json configs[2] / [3]
    "c3": dict(),
    "c4": dict(advanced_clears=True, penalise_holes_increase=True, penalise_height_increase=True),
}
KERNEL_SOURCES = ("gym-simpletetris_amd/csrc/st_kernels.hip", "gym-simpletetris_amd/csrc/st_internal.h",
                  "include/simpletetris.h")
DEBUG = os.environ.get("ST_BENCH_DEBUG") == "1"
REF_PY_STEPS_PER_S = 32752  # reference TetrisEnv.step(), 1 core of the build container


# ----------------------------------------------------------------------------- bytes
def s8d_bytes(p_lock: float, f32: bool) -> float:
    """SURVEY §8(d)'s fixed formula, bytes per env-step: 182 + 184 p_lock
    (packed obs) or 902 + 184 p_lock (float32 obs)."""
    return (902.0 if f32 else 182.0) + 184.0 * p_lock


def algorithmic_bytes(width: int, height: int, p_lock: float, f32: bool) -> float:
    """Bytes per env-step the engine's column-packed layout needs:
    102 + 167.7 p_lock at 10x20.  Always: read action 1 + piece 4 + time 4 +
    board 4W; write piece 4 + time 4 + reward 4 + done 1 + packed obs 4W
    (+ float32 obs 4WH).  Per lock: counters (score, lines, holes,
    piece_height, deaths, 7 counts, MT index) read + written 2*13*4, board
    write 4W, MT words read 8, and the amortised next MT generation
    (2 x 2,496 B read + 2,496 B written per ~476 draws) 15.7."""
    always = (1 + 4 + 4 + 4 * width) + (4 + 4 + 4 + 1 + 4 * width)
    if f32:
        always += 4 * width * height
    lock = 2 * 13 * 4 + 4 * width + 8 + 15.7
    return always + lock * p_lock


def rollout_bytes(width: int, height: int, p_lock: float, f32: bool, k: int) -> float:
    """Bytes per env-step of the K-step rollout kernel (I/O per
    step + state r/w per K steps): per step read action 1, write packed obs 4W
    + reward 4 + done 1 (+ float32 obs 4WH); per lock MT words 8 + amortised
    next generation 15.7; per launch the state (board 4W + 14 counters +
    piece) read and written once, / K."""
    step = 1 + 4 * width + 4 + 1 + (4 * width * height if f32 else 0)
    state = 2 * (4 * width + 15 * 4)
    return step + 23.7 * p_lock + state / k


# ----------------------------------------------------------------------------- PMC
def kernel_source_sha() -> str:
    """sha256 over the kernel sources: ties a PMC summary to the code it measured."""
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def step_grid(n: int) -> int:
    """Grid size in threads of k_step for n envs (two waves per 64 envs),
    part of the key tools/pmc_summary.py files a launch under."""
    return (n + 63) // 64 * 128


def image_launch(n: int, size: int, ch: int, as_u8: bool):
    """(rocprofv3 kernel name, grid size in threads) of st_grayscale's launch,
    as launch_grayscale (st_kernels.hip) picks it: float32 rgb in sweep order
    (at most 1,024 blocks of 4 waves, 4 1-KB runs per wave iteration), else
    2 envs per 256-thread block."""
    t = "unsigned char" if as_u8 else "float"
    V = 16 if as_u8 else 4
    per = size * size * ch
    if not as_u8 and ch == 3 and 64 * V * 4 <= per and (n * per) % V == 0:
        runs = (n * per + 64 * V - 1) // (64 * V)
        return f"k_grayscale_sweep<{t}, {ch}>", min((runs + 15) // 16, 1024) * 256
    return f"k_grayscale<{t}, {ch}>", (n + 1) // 2 * 256


def launch_key(kname: str, grid: int, k: int) -> str:
    """The key a profile summary files a launch under: kernel name, grid size
    in threads and steps per launch (1 for st_step, K for st_rollout), so a
    number is only ever reported beside a run of the same launch shape."""
    return f"{kname}@{grid}@k{k}"


def load_pmc(kname: str, sha: str):
    """Per-launch HBM bytes (FETCH+WRITE, gfx950-corrected by
    tools/pmc_summary.py) of `kname` (launch_key: that kernel at that grid
    size and steps per launch) from a committed profiles/*_pmc.json whose
    kernel-source hash equals the running sources'; (None, reason) if none."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if d.get("kernel_source_sha") != sha:
            continue
        v = d.get("kernels", {}).get(kname)
        if v is not None:
            return v.get("hbm_bytes_per_launch"), os.path.basename(f)
    return None, f"no PMC pass of these kernel sources (sha {sha}) at this launch shape ({kname}) under profiles/"


def load_trace(kname: str, sha: str):
    """rocprofv3 kernel-trace duration stats of `kname` (launch_key, the
    longest run of launches, with the p_lock of the traced bench run) from a
    committed profiles/*_trace.json (tools/trace_summary.py --json) of the
    same kernel sources; None if none."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_trace.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if d.get("kernel_source_sha") != sha:
            continue
        v = d.get("kernels", {}).get(kname)
        if v is not None:
            return dict(v, source=os.path.basename(f))
    return None


# ----------------------------------------------------------------------------- CPU baseline
def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds: float, config: str):
    """The C oracle (a restatement of the reference step; the Python reference
    cannot travel to the GPU box) on a bounded sample of the same workload:
    4,096 envs per process, same seeds/actions, auto-reset.  One process on one
    core, then one process per core of this process's CPU share at once;
    `value` is the aggregate.  The share: the affinity mask, capped by
    OMP_NUM_THREADS when the harness sets it (the GPU box exports 16 = its
    CPU share per GPU, while nproc / the affinity mask show all the host's
    cores, which other jobs use)."""
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--envs", "4096", "--seconds", str(seconds),
           "--config", config]

    def launch(p):
        return subprocess.Popen(cmd + ["--offset", str(p * 4096)], cwd=ROOT, stdout=subprocess.PIPE,
                                env=dict(os.environ, OMP_NUM_THREADS="1"))

    def result(pr):
        out, _ = pr.communicate()
        if pr.returncode != 0:
            raise RuntimeError(f"oracle.cpu_bench failed with {pr.returncode}")
        return json.loads(out.decode().strip().splitlines()[-1])
    one = result(launch(0))
    single = one["env_steps"] / one["seconds"]
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = avail
    try:
        share = min(avail, int(os.environ["OMP_NUM_THREADS"]))
        why = f"OMP_NUM_THREADS={share} (the harness's CPU share; affinity mask {avail})"
    except (KeyError, ValueError):
        why = f"affinity mask ({avail} cores)"
    P = max(1, share)
    rs = [result(pr) for pr in [launch(p) for p in range(P)]]
    agg = sum(r["env_steps"] / r["seconds"] for r in rs)
    return dict(value=agg, unit="env-steps/s", cores=P, kind="port",
                per_core=agg / P, single_core=single, nproc=os.cpu_count(), cores_available=avail,
                cores_basis=why, cpu_model=cpu_model(),
                sample=f"C oracle (oracle/tetris_oracle.c) on {P} processes x 4096 envs (one per core of "
                       f"the share: {why}), {rs[0]['steps']} steps each in ~{seconds:.0f} s (aggregate of "
                       f"per-process rates); 1 process alone: {single:.4g} env-steps/s ({one['steps']} steps)",
                reference_python_1core_build_container=REF_PY_STEPS_PER_S)


# ----------------------------------------------------------------------------- launcher
def rank_topology(dev, rank: int, local_rank: int, world: int, use_dist: bool, backend: str) -> dict:
    """This rank's device identity (index, name, UUID / PCI ids where torch
    exposes them), all-gathered over the process group when there is one:
    ranks_seen = the identities received, distinct_devices = the distinct
    physical GPUs among them (UUID, else PCI domain:bus:device, else host +
    visible-device list + index), and the RCCL version the nccl backend
    loaded."""
    import socket
    p = torch.cuda.get_device_properties(dev)
    ident = {"rank": rank, "local_rank": local_rank, "device_index": dev.index, "name": p.name,
             "host": socket.gethostname()}
    for k in ("uuid", "pci_domain_id", "pci_bus_id", "pci_device_id"):
        v = getattr(p, k, None)
        if v is not None:
            ident[k] = str(v)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") \
        or os.environ.get("CUDA_VISIBLE_DEVICES")
    if "uuid" in ident:
        key = "uuid:" + ident["uuid"]
    elif "pci_bus_id" in ident:
        key = "pci:%s:%s:%s" % (ident["host"], ident.get("pci_domain_id"), ident["pci_bus_id"]) \
            + ":%s" % ident.get("pci_device_id")
    else:
        key = "idx:%s:%s:%s" % (ident["host"], vis, dev.index)
    ident["device_key"] = key
    devices = [ident]
    if use_dist:
        devices = [None] * world
        dist.all_gather_object(devices, ident)
    rccl = None
    if backend == "nccl" and use_dist:
        try:
            v = torch.cuda.nccl.version()
            rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception as ex:  # noqa: BLE001 (reported, not fatal)
            rccl = f"unknown ({ex})"
    return {"ranks_seen": len(devices), "distinct_devices": distinct_devices(devices),
            "backend": backend if use_dist else None, "rccl_version": rccl, "devices": devices}


def distinct_devices(devices: list) -> int:
    """Distinct physical GPUs among the ranks' identities: the largest count
    any identity every rank reported gives -- UUIDs (all-zero ones ignored),
    then host + PCI domain:bus:device -- so that one missing or degenerate
    field cannot make distinct GPUs look shared (two ranks on one GPU agree on
    every field); the device_key alone when neither is there."""
    counts = []
    uu = [d.get("uuid") for d in devices]
    if all(u and u.strip("0-") for u in uu):
        counts.append(len(set(uu)))
    if all(d.get("pci_bus_id") is not None for d in devices):
        counts.append(len({(d.get("host"), d.get("pci_domain_id"), d["pci_bus_id"], d.get("pci_device_id"))
                           for d in devices}))
    if not counts:
        counts.append(len({d["device_key"] for d in devices}))
    return max(counts)


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly: start N rank processes (this parent
    never touches a GPU), rendezvous on 127.0.0.1, return the worst exit code."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0:
                rc = rc or r
                for q in live:  # a failed rank would leave the others in a barrier
                    q.terminate()
        time.sleep(0.05)
    return rc


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4000,
                    help="timed steps (the default spans a next-MT-generation switch of most envs)")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--obs", choices=("packed", "f32"), default="packed")
    ap.add_argument("--launch", choices=("native", "eager", "graph"), default="native",
                    help="timed steps as K st_step kernel launches enqueued by ONE st_step_n call "
                         "(native: the library's own launch loop, no Python between launches), by K "
                         "ctypes st_step calls (eager), or as one hipGraph of them (graph replay: "
                         "2.5%% slower at K=4000, profiles/r02_launch_ab.jsonl)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--gather-format", choices=("wire", "rows"), default="wire",
                    help="C5 (--gpus > 1, packed obs): what each step gathers to rank 0 -- st_step_wire's "
                         "bit stream (8 words = 32 B per 10x20 env: the obs bits, the reward's 32 bits, done; "
                         "rank 0 decodes it inside the timed region) or st_step's obs/reward/done rows (48 B)")
    ap.add_argument("--rollout-chunk", type=int, default=100, help="steps per st_rollout launch")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="headline only (profiling passes)")
    ap.add_argument("--no-clear-heavy", action="store_true")
    ap.add_argument("--no-surfaces", action="store_true",
                    help="skip the Python-surface timings (single_env, vec_env): PMC passes, whose "
                         "per-kernel averages would otherwise mix in their launches")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # ST_BENCH_SHARED_GPU=1 (tests only): every rank on cuda:0, to exercise the
    # N>1 logic on a one-GPU box with --backend gloo
    shared = os.environ.get("ST_BENCH_SHARED_GPU") == "1"
    dev_idx = 0 if shared else local_rank
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    # ST_BENCH_FORCE_DIST=1 (tests only): the torch.distributed path (RCCL with
    # the nccl backend) even at one rank, so a one-GPU box runs its calls
    use_dist = world > 1 or os.environ.get("ST_BENCH_FORCE_DIST") == "1"
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from gym_simpletetris_amd import _lib as C
    from gym_simpletetris_amd.distributed import ShardedTetris, output_buffer, buffer_views

    # which device every rank runs on, gathered over the process group (RCCL
    # with the nccl backend), so the driver's N-GPU record shows that the
    # collective formed an N-rank communicator over N distinct GPUs
    topo = rank_topology(dev, rank, local_rank, world, use_dist, args.backend)
    if use_dist and topo["distinct_devices"] != world and not shared:
        raise SystemExit(f"bench: {world} ranks but {topo['distinct_devices']} distinct devices: "
                         f"{topo['devices']} (set ST_BENCH_SHARED_GPU=1 only for tests that share one GPU)")

    W, H = 10, 20
    K, WU = args.steps, args.warmup
    aseed = 0x5EED
    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    sha = kernel_source_sha()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):  # an event's first record is slow (~100 us): not inside a timed region
        ev0.record(s)
        ev1.record(s)

    def sync_all():
        torch.cuda.synchronize(dev)
        if use_dist:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if not use_dist:
            return x
        if args.backend == "nccl":
            t = torch.tensor([x], dtype=torch.float64, device=dev)
        else:
            t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    pl_bufs = {}

    def spawned_dev(eng, slot: int = 0) -> torch.Tensor:
        """The envs' total spawn count (every lock spawns one piece) as a
        device scalar in slot `slot` of a per-engine result pair, computed on
        s (no host wait) into buffers allocated at the engine's first call --
        Workload.__init__, before the warm-up: a device allocation (or a
        torch kernel's first use) right before the timed region made its
        first st_step call cost ~20 us of host time (profiles/r05/
        region_probe_*.jsonl).  (A pinned-host copy summed on the host instead
        measured 4% slower at the driver's K = 20 -- 1.17 against 1.22e10,
        profiles/r05/ab_k20_counter_read.txt -- though it sped the rollout
        line up 1.30 -> 1.27-1.30 us/step.)"""
        bufs = pl_bufs.get(id(eng))
        if bufs is None:
            bufs = pl_bufs[id(eng)] = (torch.empty((7, eng.stride), dtype=torch.int32, device=dev),
                                       torch.zeros(2, dtype=torch.int64, device=dev))
        cnt, res = bufs
        src = eng._views.stats + C.STAT["count0"] * eng.stride * 4  # rows count0 .. count0 + 6
        C.check(eng._L.st_copy(ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(src), cnt.numel() * 4, sp))
        torch.sum(cnt[:, :eng.n], dim=(0, 1), dtype=torch.int64, out=res[slot])
        return res[slot]

    def timed(eng, run, nsteps):
        """Time `run()` (enqueues exactly nsteps steps of `eng` on s): barrier +
        synchronize on both sides, max over ranks; events on s give the GPU
        span.  p_lock from the spawn counters (every lock spawns one piece),
        summed on s after everything enqueued before the region and read
        after it (no blocking host read between the warm-up and the region:
        a thread that just slept in a long wait issues its next launches
        slowly: round 4's k20_idle / k20_sync probes, in git history)."""
        with torch.cuda.stream(s):  # s is current for the whole region (graph replay launches on it)
            c0 = spawned_dev(eng, 0)
            ev0.record(s)  # first host calls after a stream switch are slow: not inside the region
            ev1.record(s)
            sync_all()
            # the start event is recorded on the idle stream right before the
            # region's clock starts (its host call is instrumentation, not a
            # step: round 3 had it inside the region); the end event goes in
            # right behind the K launches, while the GPU is still running them
            ev0.record(s)
            t0 = t1 = time.perf_counter()
            run()
            t2 = time.perf_counter()
            ev1.record(s)
            t3 = time.perf_counter()
            sync_all()
            t4 = time.perf_counter()
        elapsed = max_over_ranks(t4 - t0)
        with torch.cuda.stream(s):  # (the read on s too: c0 / c1 were computed there)
            c1 = spawned_dev(eng, 1)
            n_sp = int((c1 - c0).item())
        if DEBUG:
            print("timed: rec0 %.1f run %.1f rec1 %.1f sync %.1f us" % ((t1 - t0) * 1e6, (t2 - t1) * 1e6,
                  (t3 - t2) * 1e6, (t4 - t3) * 1e6), file=sys.stderr)
        p_lock = n_sp / float(eng.n * nsteps)
        return elapsed, ev0.elapsed_time(ev1), p_lock

    def make_actions(n, offset, gen):
        a = torch.empty((WU + K, n), dtype=torch.uint8, device=dev)
        for t in range(WU + K):
            gen(t, aseed, global_offset=offset, out=a[t])
        return a

    cus = torch.cuda.get_device_properties(dev).multi_processor_count

    def rollout_three_wave(n):
        """launch_rollout's choice: the three-wave kernel up to 4 workgroups
        (of 64 envs) per CU, else the two-wave one."""
        return (n + 63) // 64 <= 4 * cus

    def kname_of(kind, f32, sc0, n=None):  # rocprofv3's demangled name of the 10x20 kernel
        b = lambda v: "true" if v else "false"  # noqa: E731
        if kind == "step":
            return f"k_step<10, 20, {b(f32)}, false, {b(sc0)}, false>"
        if rollout_three_wave(n):
            return f"k_rollout<10, 20, {b(f32)}, {b(sc0)}, false>"
        return f"k_rollout2<10, 20, {b(f32)}, {b(sc0)}>"

    def rollout_grid(n):
        return (n + 63) // 64 * (192 if rollout_three_wave(n) else 128)

    def roofline(ev_us, bpe, units_per_launch, kname, extra=None, grid=None, k=1, bytes_at=None):
        """Roofline object of one launch shape: `achieved` = algorithmic bytes
        per launch / the HIP-event time per launch of the timed region (the
        contract's live measurement; at small K it includes the region's ramp);
        `traffic` and `rocprof` only from committed profiles of the same
        kernel sources AND launch shape (kernel, grid, steps per launch),
        else null with the reason.  bytes_at(p_lock) re-prices the bytes at
        the traced run's own p_lock for the rocprof fraction."""
        bpl = bpe * units_per_launch
        achieved = bpl / (ev_us * 1e-6) / 1e9
        key = launch_key(kname, grid, k) if grid is not None else None
        if key is None:
            traffic, src = None, "not collected for this variant"
        else:
            traffic, src = load_pmc(key, sha)
        r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": achieved / HBM_PEAK_GBS,
             "frac_basis": "bytes_per_launch / (HIP-event span of the timed region / launches)",
             "traffic": traffic, "kernel": kname, "launch_key": key,
             "event_us_per_launch": ev_us, "bytes_per_env_step": bpe, "bytes_per_launch": bpl,
             "traffic_source": src, "kernel_source_sha": sha}
        tr = load_trace(key, sha) if key is not None else None
        if tr is not None:  # the committed rocprofv3 trace of the same sources and launch shape
            pl = tr.get("p_lock")
            bpl_tr = bytes_at(pl) * units_per_launch if (bytes_at and pl is not None) else bpl
            r["rocprof"] = {"mean_us": tr["mean_us"], "median_us": tr["median_us"],
                            "launches": tr["launches"], "source": f"{tr['source']} ({tr['trace']})",
                            "p_lock_traced_run": pl, "bytes_per_launch_traced_run": bpl_tr,
                            "frac_at_traced_mean": bpl_tr / (tr["mean_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS,
                            "frac_at_traced_median": bpl_tr / (tr["median_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS}
        if extra:
            r.update(extra)
        return r

    def action_rows(eng_gen, offset, n, t0, T, have):
        """Action rows t0 .. t0+T-1 of the synthetic stream for this shard: a
        slice of `have` (rows 0..len-1) when it holds them, else generated."""
        if have is not None and t0 + T <= have.shape[0]:
            return have[t0:t0 + T]
        a = torch.empty((T, n), dtype=torch.uint8, device=dev)
        for t in range(T):
            eng_gen(t0 + t, aseed, global_offset=offset, out=a[t])
        return a

    class Workload:
        """One engine shard + its K+W action rows + reused output buffers."""

        def __init__(self, n_local, cfg_kw, f32):
            n_global = n_local * world
            self.sh = ShardedTetris(n_global, seed=1000, rank=rank, world=world, device=dev,
                                    autoreset="same_step", width=W, height=H, **cfg_kw)
            self.eng = self.sh.engine
            self.n_local, self.n_global = n_local, n_global
            self.sc0 = not cfg_kw  # no scoring flags: the SC0 kernel specialization
            self.f32 = f32
            self.actions = make_actions(n_local, self.sh.offset, self.eng.gen_actions)
            self.eng.reset()
            torch.cuda.synchronize(dev)  # reset + actions (current stream) before s uses them
            with torch.cuda.stream(s):  # the spawn counter's buffers and kernels, before any timing
                spawned_dev(self.eng, 0)
            # region_probe's events, created and first recorded now (a first
            # record costs ~100 us of host time; creating them right before a
            # region slowed its first launch)
            self.pevs = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)] if K <= 200 else []
            with torch.cuda.stream(s):
                for e_ in self.pevs:
                    e_.record(s)
            torch.cuda.synchronize(dev)
            self.obs_f32 = torch.zeros((n_local, W, H), dtype=torch.float32, device=dev) if f32 else None
            self.ptrs = [ctypes.c_void_p(x.data_ptr()) for x in (self.sh._obs, self.sh._rew, self.sh._done)]
            self.pf = ctypes.c_void_p(self.obs_f32.data_ptr()) if f32 else None
            self.aptr = [ctypes.c_void_p(self.actions[t].data_ptr()) for t in range(WU + K)]
            L, ctx = self.eng._L, self.eng._ctx
            po, pr, pd = self.ptrs
            # the ctypes argument tuple of every step, built once: the timed
            # loop is one ctypes call per step and nothing else (return codes
            # OR'ed, checked after the loop) -- the HIP runtime's own launch
            # cost (~3.2 us, tools/launch_cost.hip) is then the host's whole
            # share, under the kernel's ~4.7 us
            if f32:
                self.fn = L.st_step_f32
                self.args = [(ctx, self.aptr[t], po, self.pf, pr, pd, sp) for t in range(WU + K)]
            else:
                self.fn = L.st_step
                self.args = [(ctx, self.aptr[t], po, pr, pd, sp) for t in range(WU + K)]
            # --launch native: every step's action pointer in one host array,
            # so K steps are one st_step_n call (K kernel launches from C)
            self.aarr = (ctypes.c_void_p * (WU + K))(*[a.value for a in self.aptr])
            self.nargs = (ctx, po, self.pf, pr, pd, sp)

        def launch(self, t):
            C.check(self.fn(*self.args[t]))

        def launch_range(self, t0, t1):
            """Steps t0 .. t1-1: one st_step kernel launch each, enqueued by
            one st_step_n call (--launch native) or one ctypes st_step call
            per step (eager; graph capture)."""
            if args.launch == "native":
                ctx, po, pf, pr, pd, sp_ = self.nargs
                C.check(self.eng._L.st_step_n(ctx, ctypes.addressof(self.aarr) + t0 * ctypes.sizeof(ctypes.c_void_p),
                                              t1 - t0, po, pf, pr, pd, sp_))
                return
            fn, rc = self.fn, 0
            for a in self.args[t0:t1]:
                rc = rc or fn(*a)  # stop at the first failure and report its code
            C.check(rc)

        def warmup(self):
            with torch.cuda.stream(s):
                self.launch_range(0, WU)
            torch.cuda.synchronize(dev)

        # ---- BASELINE C5: every step's outputs gathered to rank 0 ----
        def setup_gather(self):
            """Two output buffers -- st_step_wire's [words][n] rows (the
            default with packed obs) or st_step's [W+2][n] packed obs | reward
            | done (distributed.output_buffer) -- rank 0's receive lists, and
            the ctypes arguments of every step writing into buffer t % 2."""
            self.nccl = args.backend == "nccl"
            self.wire = args.gather_format == "wire" and not self.f32
            if self.wire:
                self.gbufs = [torch.zeros((self.eng.wire_words, self.n_local), dtype=torch.int32, device=dev)
                              for _ in range(2)]
                self.gfn = self.eng._L.st_step_wire
            else:
                self.gbufs = [output_buffer(W, self.n_local, dev) for _ in range(2)]
                self.gfn = self.fn
                views = [[ctypes.c_void_p(v.data_ptr()) for v in buffer_views(b, W)] for b in self.gbufs]
            rdev = dev if self.nccl else torch.device("cpu")  # gloo gathers host tensors
            # rank 0 receives each step into one contiguous [world][rows][n]
            # buffer (per step parity), gathered into its views
            self.grecv_buf = [torch.empty((world,) + tuple(b.shape), dtype=b.dtype, device=rdev)
                              if rank == 0 else None for b in self.gbufs]
            self.grecv = [list(rb.unbind(0)) if rb is not None else None for rb in self.grecv_buf]
            # rank 0's decoded global outputs of every step (wire: st_unwire_shards
            # of the receive buffer, inside the timed region): obs [W][N], reward, done
            if rank == 0 and self.wire:
                self.gout = (torch.empty((W, self.n_global), dtype=torch.int32, device=dev),
                             torch.empty(self.n_global, dtype=torch.int32, device=dev),
                             torch.empty(self.n_global, dtype=torch.bool, device=dev))
                self.gdec = (ctypes.c_void_p(self.gout[0].data_ptr()), ctypes.c_void_p(self.gout[1].data_ptr()),
                             ctypes.c_void_p(self.gout[2].data_ptr()))
                self.grecv_dev = [rb if self.nccl else torch.empty(rb.shape, dtype=rb.dtype, device=dev)
                                  for rb in self.grecv_buf]
            self.decode = True
            self.ndecodes = 0
            ctx = self.eng._ctx
            if self.wire:
                self.gargs = [(ctx, self.aptr[t], ctypes.c_void_p(self.gbufs[t & 1].data_ptr()), sp)
                              for t in range(WU + K)]
            elif self.f32:
                self.gargs = [(ctx, self.aptr[t], views[t & 1][0], self.pf, views[t & 1][1], views[t & 1][2], sp)
                              for t in range(WU + K)]
            else:
                self.gargs = [(ctx, self.aptr[t], *views[t & 1], sp) for t in range(WU + K)]
            self.gworks = [None, None]
            self.ngathers = 0

        def decode_step(self, k):
            """Rank 0, wire format: st_unwire_shards of step parity k's
            receive buffer into the global obs / reward / done (on s, after
            the gather that filled it: its work was waited on s)."""
            src = self.grecv_dev[k]
            if not self.nccl:  # gloo: the host receive buffer to the GPU first
                src.copy_(self.grecv_buf[k], non_blocking=False)
            rc = self.eng._L.st_unwire_shards(W, H, self.n_global, world, self.n_local, ctypes.c_void_p(src.data_ptr()),
                                   *self.gdec, sp)
            self.ndecodes += 1
            return rc

        def gather_range(self, t0, t1):
            """Steps t0 .. t1-1, each one st_step into buffer t % 2 and one
            gather of that buffer to rank 0.  With RCCL the gather runs on
            the collective's stream after the step (ProcessGroupNCCL orders
            it behind the current stream, s), so step t+1 overlaps the gather
            of step t; before step t+2 reuses a buffer, s waits for the gather
            that read it.  With the wire format and self.decode, rank 0
            decodes every step's gathered outputs into the global obs /
            reward / done (BASELINE C5's deliverable) one step later: after
            step t+1 is enqueued, s waits for the gather of step t and runs
            st_unwire_shards on it, so the gather of step t still overlaps
            step t+1.  All gathers (and decodes) are complete on s when this
            returns."""
            fn, rc = self.gfn, 0
            dec = self.decode and self.wire and rank == 0
            pend = None  # step parity whose gather rank 0 has yet to decode
            for t in range(t0, t1):
                k = t & 1
                if self.gworks[k] is not None:
                    self.gworks[k].wait()  # s (not the host) waits for the gather of step t - 2
                    self.gworks[k] = None
                rc = rc or fn(*self.gargs[t])
                if dec and pend is not None:
                    if self.gworks[pend] is not None:
                        self.gworks[pend].wait()  # s waits for the gather of step t - 1
                        self.gworks[pend] = None
                    rc = rc or self.decode_step(pend)
                    pend = None
                if self.nccl:
                    self.gworks[k] = dist.gather(self.gbufs[k], gather_list=self.grecv[k], dst=0, async_op=True)
                else:  # gloo: through host memory, no overlap
                    s.synchronize()
                    dist.gather(self.gbufs[k].cpu(), gather_list=self.grecv[k], dst=0)
                self.ngathers += 1
                pend = k
            for k in (0, 1):
                if self.gworks[k] is not None:
                    self.gworks[k].wait()
                    self.gworks[k] = None
            if dec and pend is not None:
                rc = rc or self.decode_step(pend)
            C.check(rc)

        def measure_gather(self):
            """C5's timed region: K x (st_step + gather to rank 0 + rank 0's
            decode of the gathered wire rows into the global obs / reward /
            done) after WU such steps untimed; then the same K steps without
            the decode, reported beside (`no_decode`).  Rank 0's decoded
            outputs of the last timed step go to $ST_BENCH_DUMP (an .npz)
            when set (tests compare them with the oracle)."""
            self.setup_gather()
            with torch.cuda.stream(s):
                self.gather_range(0, WU)
            torch.cuda.synchronize(dev)
            g0, d0 = self.ngathers, self.ndecodes
            el, ev_ms, p_lock = timed(self.eng, lambda: self.gather_range(WU, WU + K), K)
            ng, nd = self.ngathers - g0, self.ndecodes - d0
            dump = os.environ.get("ST_BENCH_DUMP")
            if rank == 0 and dump:
                import numpy as np
                from gym_simpletetris_amd.distributed import assemble
                if self.wire:  # the region's own last decode (st_unwire_shards)
                    torch.cuda.synchronize(dev)
                    o, r, d = (x.cpu() for x in self.gout)
                else:
                    got = self.grecv[(WU + K - 1) & 1]
                    o, r, d = assemble([b.cpu() for b in got], W)
                np.savez(dump, obs=o.numpy().view(np.uint32), reward=r.numpy(), done=d.numpy(),
                         step=WU + K - 1, n_global=self.n_global, gathers_timed=ng, decodes_timed=nd)
            bpr = self.gbufs[0].numel() * 4
            ms = el / K * 1e3
            out = {"value": self.n_global * K / el, "ms_per_step": ms, "event_ms_per_step": ev_ms / K,
                   "p_lock": p_lock, "gathers_timed": ng,
                   "gather": {"backend": args.backend, "collective": "torch.distributed.gather to rank 0",
                              "format": ("st_step_wire: %d words per env (obs bits, reward 32 bits, done)"
                                         % self.eng.wire_words if self.wire else
                                         "st_step rows: packed obs [W] + reward + done per env"),
                              "gathers_in_timed_region": ng, "decodes_in_timed_region_rank0": nd,
                              "decode": ("rank 0: st_unwire_shards of each step's receive buffer into the "
                                         "global obs [W][N] / reward / done, on the step stream, inside the "
                                         "region" if self.wire else "none (the rows are st_step's outputs)"),
                              "bytes_per_rank_per_step": bpr,
                              "bytes_into_rank0_per_step": bpr * (world - 1),
                              "rank0_ingress_GBps": bpr * (world - 1) / (ms * 1e-3) / 1e9,
                              "overlap": "double-buffered: step t+1 computes while step t is gathered"}}
            if self.wire:
                self.decode = False
                el2, ev2, _ = timed(self.eng, lambda: self.gather_range(WU, WU + K), K)
                self.decode = True
                out["gather"]["no_decode"] = {"value": self.n_global * K / el2, "ms_per_step": el2 / K * 1e3,
                                    "event_ms_per_step": ev2 / K,
                                    "basis": "the same K steps + gathers again, rank 0 not decoding"}
            return out

        def runner(self):
            if args.launch != "graph":
                return (lambda: self.launch_range(WU, WU + K)), None
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self.launch_range(WU, WU + K)
            torch.cuda.synchronize(dev)
            return g.replay, g

        def steady(self, S=1000):
            """After the timed region: S more launches back to back (action
            rows reused cyclically), HIP events around them only -- the
            kernel's launch-to-launch period without the region's ramp (the
            first launch after an idle GPU, the final synchronize)."""
            def run():
                done = 0
                while done < S:
                    c = min(K, S - done)
                    self.launch_range(WU, WU + c)
                    done += c
            el, ev_ms, p_lock = timed(self.eng, run, S)
            return ev_ms * 1e3 / S, p_lock

        def region_probe(self):
            """Debug record of the timed region's shape (outside `value`): the
            same K eager launches run twice more right after the region, from
            the same idle-GPU start (barrier + synchronize): (1) with a host
            perf_counter stamp after every launch call and HIP events only
            around the region -- the host's submission timeline, unperturbed;
            (2) with a HIP event recorded before every launch -- each launch's
            GPU span (the events add host time per launch, so the host falls
            behind the GPU sooner than in the region: read its shape, not its
            sum)."""
            evs = self.pevs  # created and first recorded in __init__
            fn, args_ = self.fn, self.args[WU:WU + K]
            out = {}
            with torch.cuda.stream(s):
                # the timed region's own prelude (spawn count, event records)
                spawned_dev(self.eng, 0)
                ev0.record(s)
                ev1.record(s)
                sync_all()
                ev0.record(s)
                t0 = time.perf_counter()
                hs = []
                for a in args_:
                    fn(*a)
                    hs.append(time.perf_counter())
                ev1.record(s)
                sync_all()
                t1 = time.perf_counter()
                out["host_submit_us"] = [round((h - t0) * 1e6, 2) for h in hs]
                out["host_call_us"] = [round((b_ - a_) * 1e6, 2) for a_, b_ in zip([t0] + hs[:-1], hs)]
                out["wall_us"] = round((t1 - t0) * 1e6, 1)
                out["event_span_us"] = round(ev0.elapsed_time(ev1) * 1e3, 2)
                out["sync_after_last_submit_us"] = round((t1 - hs[-1]) * 1e6, 1)
                spawned_dev(self.eng, 0)
                sync_all()
                t0 = time.perf_counter()
                for i, a in enumerate(args_):
                    evs[i].record(s)
                    fn(*a)
                evs[K].record(s)
                sync_all()
                t1 = time.perf_counter()
                out["per_launch_event_us"] = [round(evs[i].elapsed_time(evs[i + 1]) * 1e3, 2) for i in range(K)]
                out["events_wall_us"] = round((t1 - t0) * 1e6, 1)
            out["basis"] = ("the timed region's K launches repeated twice after it (same actions, later "
                            "state): host stamps only, then an event before every launch; debug, not value")
            return out

        def measure(self, steady=True):
            self.warmup()
            run, keep = self.runner()
            el, ev_ms, p_lock = timed(self.eng, run, K)
            del keep
            probe = self.region_probe() if (steady and K <= 200 and args.launch == "eager") else None
            ev_us = ev_ms * 1e3 / K
            kname = kname_of("step", self.f32, self.sc0)
            bytes_at = lambda pl: s8d_bytes(pl, self.f32)  # noqa: E731
            rl = roofline(ev_us, s8d_bytes(p_lock, self.f32), self.n_local, kname, grid=step_grid(self.n_local),
                          k=1, bytes_at=bytes_at, extra={
                "bytes_formula": "SURVEY 8(d): %d + 184 p_lock" % (902 if self.f32 else 182),
                "bytes_per_env_step_layout": algorithmic_bytes(W, H, p_lock, self.f32),
                "frac_layout": algorithmic_bytes(W, H, p_lock, self.f32) * self.n_local
                / (ev_us * 1e3) / HBM_PEAK_GBS,
                "p_lock": p_lock})
            if rl["traffic"] is not None:
                rl["traffic_over_layout_bytes"] = rl["traffic"] / (rl["bytes_per_env_step_layout"] * self.n_local)
            if steady:
                st_us, st_pl = self.steady()
                rl["steady"] = {"launches": 1000, "event_us_per_launch": st_us, "p_lock": st_pl,
                                "frac": s8d_bytes(st_pl, self.f32) * self.n_local / (st_us * 1e3) / HBM_PEAK_GBS,
                                "basis": "1,000 further launches back to back after the timed region, "
                                         "HIP events around them (no region ramp / final synchronize)"}
            r = {"value": self.n_global * K / el, "ms_per_step": el / K * 1e3,
                 "event_ms_per_step": ev_ms / K, "p_lock": p_lock, "roofline": rl}
            if probe is not None:
                r["region_probe"] = probe
            return r

        def close(self):
            self.eng.close()

    cfg_kw = CONFIGS[args.config]
    f32 = args.obs == "f32"
    head = Workload(args.n_envs, cfg_kw, f32)
    if use_dist:
        # BASELINE C5: each timed step = st_step on every shard + the gather
        # of its outputs to rank 0; the same steps without the gather beside it
        gm = head.measure_gather()
        ng = head.measure(steady=False)
        hm = dict(gm, roofline=dict(ng["roofline"], note="st_step, the engine's kernel, from the "
                                    "gather-free steps (step_no_gather); the gather's rate is in `gather`"))
    else:
        hm = head.measure()
    out = {
        "metric": METRIC,
        "value": hm["value"],
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": WU,
        "ms_per_step": hm["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (uniform splitmix64 actions, seeds 1000 + global env index)",
        "config": {
            "workload": (f"C5: {head.n_global} boards sharded {args.n_envs} per GPU x {world}, one st_step per "
                         f"shard per step + a gather of its obs/reward/done to rank 0 per step "
                         f"({'st_step_wire bit stream' if args.gather_format == 'wire' and not f32 else 'rows'}), "
                         if use_dist else
                         f"{args.config.upper()}: {args.n_envs} parallel {W}x{H} boards per GPU, one "
                         f"st_step per step, ")
                        + f"ram obs ({args.obs}), auto-reset, "
                        + ("advanced_clears+penalise_holes_increase+penalise_height_increase"
                           if args.config == "c4" else "default rewards"),
            "envs_per_gpu": args.n_envs,
            "envs_total": head.n_global,
            "board": f"{W}x{H}",
            "obs": args.obs,
            "launch": {"graph": "hipGraph of K st_step launches",
                       "eager": "K eager st_step launches, one ctypes call each",
                       "native": "K st_step launches enqueued by one st_step_n call (the library's launch loop)"}[
                args.launch],
            "parallelism": f"env-shard x{world}",
            "hip_force_dev_kernarg": os.environ.get("HIP_FORCE_DEV_KERNARG"),
            "hip_force_dev_kernarg_from": "environment" if KERNARG_FROM_ENV else "bench.py (tune_runtime opt-in)",
        },
        "p_lock": hm["p_lock"],
        "event_ms_per_step": hm["event_ms_per_step"],
        "roofline": hm["roofline"],
        "ranks_seen": topo["ranks_seen"],
        "distinct_devices": topo["distinct_devices"],
        "rccl_version": topo["rccl_version"],
        "topology": topo,
    }
    if "region_probe" in hm:
        out["debug"] = {"region_probe": hm["region_probe"]}
    if use_dist:
        out["gather"] = hm["gather"]
        out["config"]["gathers_per_step"] = 1
        out["step_no_gather"] = {k: ng[k] for k in ("value", "ms_per_step", "event_ms_per_step", "p_lock")}

    if not args.no_extras:
        variants = {}
        eng = head.eng
        L, ctx = eng._L, eng._ctx
        if not f32:  # the same st_step with the reference's float32 obs fused in
            w = Workload(args.n_envs, cfg_kw, True)
            variants["step_f32"] = w.measure(steady=False)
            w.close()
        # K-step rollout kernel (st_rollout), continuing the headline's state:
        # a fixed CH steps per launch whatever K is (so its PMC / trace keys
        # match the profiles' launch shape), max(5, K // CH) timed launches
        # (at the driver's K = 20 a single launch would carry the region's
        # fixed ~40 us alone)
        CH = args.rollout_chunk
        nch = max(5, K // CH)
        n_local = head.n_local
        ro = torch.empty((CH, W, n_local), dtype=torch.int32, device=dev)
        rr = torch.empty((CH, n_local), dtype=torch.int32, device=dev)
        rd = torch.empty((CH, n_local), dtype=torch.uint8, device=dev)
        racts = action_rows(eng.gen_actions, head.sh.offset, n_local, WU, (nch + 1) * CH, head.actions)
        for use_f32 in (False, True):
            rf = torch.empty((CH, n_local, W, H), dtype=torch.float32, device=dev) if use_f32 else None
            aptr = [ctypes.c_void_p(racts[c * CH].data_ptr()) for c in range(nch + 1)]
            ptrs = [ctypes.c_void_p(x.data_ptr()) if x is not None else None for x in (ro, rf, rr, rd)]

            per_launch = os.environ.get("ST_BENCH_RO_PERLAUNCH") == "1"
            pev = [torch.cuda.Event(enable_timing=True) for _ in range(nch + 1)] if per_launch else None
            if per_launch:
                with torch.cuda.stream(s):
                    for e in pev:
                        e.record(s)

            def run_ro():
                if per_launch:  # (diagnostic) an event behind every launch of the region
                    pev[0].record(s)
                for c in range(1, nch + 1):
                    C.check(L.st_rollout(ctx, CH, aptr[c], *ptrs, sp))
                    if per_launch:
                        pev[c].record(s)
            with torch.cuda.stream(s):  # warm-up launch (timed() waits for it before reading counters)
                C.check(L.st_rollout(ctx, CH, aptr[0], *ptrs, sp))
            el, ev, pl = timed(eng, run_ro, nch * CH)
            ev_us = ev * 1e3 / nch
            if per_launch:
                print(("ro_per_launch f32" if use_f32 else "ro_per_launch") + " us/step " + " ".join("%.3f" % (pev[c - 1].elapsed_time(pev[c]) * 1e3 / CH)
                                                        for c in range(1, nch + 1)), file=sys.stderr)
            variants["rollout_f32" if use_f32 else "rollout_packed"] = {
                "value": head.n_global * nch * CH / el, "ms_per_step": el / (nch * CH) * 1e3,
                "steps_per_launch": CH, "launches": nch, "p_lock": pl,
                "roofline": roofline(ev_us, rollout_bytes(W, H, pl, use_f32, CH), CH * n_local,
                                     kname_of("rollout", use_f32, head.sc0, n_local), grid=rollout_grid(n_local), k=CH,
                                     bytes_at=lambda q, f=use_f32: rollout_bytes(W, H, q, f, CH), extra=
                                     {"bytes_formula": "rollout: I/O per step + state r/w per launch / K",
                                      "p_lock": pl})}
            del rf
            if not use_f32 and os.environ.get("ST_BENCH_RO_PROBE") == "1":
                # (diagnostic) the same launches timed harness-style: HIP
                # events around 10 back-to-back launches, no timed() prelude
                pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(s):
                    C.check(L.st_rollout(ctx, CH, aptr[0], *ptrs, sp))
                    if os.environ.get("ST_BENCH_RO_PROBE_SYNC") == "1":
                        sync_all()
                    pe0.record(s)
                    for c in range(1, 11):
                        C.check(L.st_rollout(ctx, CH, aptr[c % (nch + 1)], *ptrs, sp))
                    pe1.record(s)
                torch.cuda.synchronize()
                print("ro_probe harness-style us/step %.3f" % (pe0.elapsed_time(pe1) * 1e3 / (10 * CH)), file=sys.stderr)
        del racts
        # the other single-GPU BASELINE configs: C2 (4,096 boards), C4 / C3
        other = "c3" if args.config == "c4" else "c4"
        w = Workload(args.n_envs, CONFIGS[other], f32)
        variants[other] = w.measure(steady=False)
        variants[other]["config"] = f"{other.upper()} at {args.n_envs} boards per GPU"
        w.close()
        w = Workload(4096, cfg_kw, f32)
        variants["c2"] = w.measure(steady=False)
        variants["c2"]["config"] = f"C2: 4096 boards per GPU, {args.config.upper()} rewards"
        w.close()
        variants.update(image_variants(head, C, timed, roofline, dev, s, sp, W, WU, K))
        if world == 1 and not args.no_surfaces:
            variants["single_env"] = single_env_variant(2000)
            variants["vec_env"] = vec_env_variant(args.n_envs, 1000, dev)
        if not args.no_clear_heavy and not f32:
            variants["step_clear_heavy"] = clear_heavy(head, cfg_kw, C, ShardedTetris, timed, roofline,
                                                       kname_of, dev, s, sp, rank, world, W, H, K, WU,
                                                       aseed, args.config, args.launch)
        out["variants"] = variants
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.config)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


def single_env_variant(steps: int):
    """The single-env drop-in (TetrisEnv, tetris_env.py:338-467): wall time
    per TetrisEnv.step() on uniform random actions with reset on done, numpy
    obs on the host each step, beside the reference's 30.5 us/step (SURVEY
    §6, one core of the build container; it cannot run on the GPU box)."""
    import random
    from gym_simpletetris_amd.envs.tetris_env import TetrisEnv
    out = {}
    rnd = random.Random(1)
    acts = [rnd.randrange(7) for _ in range(steps + 200)]
    for obs_type in ("ram", "grayscale"):
        for rng in ("global", "private"):
            env = TetrisEnv(obs_type=obs_type, rng=rng, seed=0)
            env.reset()
            for a in acts[:200]:
                if env.step(a)[2]:
                    env.reset()
            t0 = time.perf_counter()
            for a in acts[200:]:
                if env.step(a)[2]:
                    env.reset()
            dt = time.perf_counter() - t0
            out[f"{obs_type}/{rng}"] = {"us_per_step": dt / steps * 1e6, "steps_per_s": steps / dt}
            env.close()
    out["reference_us_per_step"] = {"ram": 1e6 / REF_PY_STEPS_PER_S, "grayscale": 1e6 / 8052,
                                    "note": "reference TetrisEnv.step(), 1 core of the build container "
                                            "(SURVEY §6), incl. reset on done"}
    return out


def vec_env_variant(n: int, steps: int, dev):
    """The batched Python surface (TetrisVecEnv.step, the vector counterpart
    of tetris_env.py:397-403) with actions already on the GPU, as an RL loop
    calls it: wall time per step, packed and float32 obs, without the action
    check, with the step kernel's own check ('async', the default: a sticky
    flag in mapped host memory, st_set_action_flag; no extra launch, no sync)
    and with the reference's immediate check (True: the action gate,
    st_gate_actions, the host waiting for the check kernel only); copy=True (default)
    and, with 'async', copy=False, and copy=True with every step's outputs
    kept for 8 steps (`/held8`: no slot is free to reuse)."""
    from gym_simpletetris_amd.envs.tetris_env import TetrisVecEnv
    out = {}
    for fmt in ("packed", "f32"):
        for val, cp, hold in ((False, True, 0), ("async", True, 0), (True, True, 0), ("async", False, 0),
                              ("async", True, 8)):
            v = TetrisVecEnv(n, seed=1000, obs_format=fmt, validate_actions=val, device=dev, copy=cp)
            v.reset()
            acts = torch.randint(0, 7, (64, n), dtype=torch.uint8, device=dev)
            ring = [None] * max(hold, 1)
            for t in range(50):
                ring[t % len(ring)] = v.step(acts[t % 64]) if hold else None
            torch.cuda.synchronize(dev)
            r0 = v.slots_reused
            t0 = time.perf_counter()
            if hold:
                for t in range(steps):
                    ring[t % hold] = v.step(acts[t % 64])
            else:
                for t in range(steps):
                    v.step(acts[t % 64])
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / steps
            key = f"{fmt}/validate_actions={val}" + ("" if cp else "/copy=False") + (f"/held{hold}" if hold else "")
            out[key] = {"us_per_step": dt * 1e6, "env_steps_per_s": n / dt}
            if cp:
                out[key]["slots_reused"] = v.slots_reused - r0
            del ring
            v.close()
    out["note"] = ("TetrisVecEnv.step incl. the per-step info snapshot; copy=True (the default): every "
                   "step's outputs in tensors of their own, never written again while the caller holds "
                   "any of them (a recent step's slot is reused once nothing of it is referenced: "
                   "slots_reused); copy=False: two alternating output slots (overwritten two steps "
                   "later); held8: copy=True with each step's outputs kept 8 steps (the slot pool "
                   "follows the holding depth: 9 slots, reused in turn); validate_actions=True: the "
                   "action gate (st_gate_actions + the gated step, the host waiting for the check "
                   "kernel only); host-bound above the kernel (DESIGN.md §5.1)")
    return out


def image_variants(head, C, timed, roofline, dev, s, sp, W, WU, K):
    """obs_type='grayscale' / 'rgb' (tetris_env.py:76-122, :426-433): the
    84x84 float32 image of every env per step (st_grayscale on st_step's
    packed obs).  Timed two ways: the image kernel alone on one packed obs
    (its roofline: reads 4W B + writes 84*84*ch*4 B per env), and whole steps
    (st_step + st_grayscale per step)."""
    eng = head.eng
    L, ctx = eng._L, eng._ctx
    n = head.n_local
    KG = max(1, min(K, 200))
    out = {}
    po, pr, pd = head.ptrs
    for name, ch in (("grayscale_f32", 1), ("rgb_f32", 3)):
        img = torch.empty((n, 84, 84, ch), dtype=torch.float32, device=dev)
        pi = ctypes.c_void_p(img.data_ptr())

        def run_img():
            for _ in range(KG):
                C.check(L.st_grayscale(ctx, po, 84, ch, 0, pi, sp))
        with torch.cuda.stream(s):
            run_img()
        el, ev, _ = timed(eng, run_img, KG)
        kern_us = ev * 1e3 / KG
        bpe = 4 * W + 84 * 84 * ch * 4
        kname, grid = image_launch(n, 84, ch, False)
        r = {"kernel_only": True, "launches": KG, "kernel_us": kern_us,
             "roofline": roofline(kern_us, bpe, n, kname,
                                  {"bytes_formula": f"read packed obs 4W + write 84*84*{ch}*4 per env"},
                                  grid=grid)}
        # whole steps with this obs_type: st_step + the image per step
        KS = max(1, min(K, 100))

        def run_steps():
            for t in range(WU, WU + KS):
                C.check(L.st_step(ctx, head.aptr[t], po, pr, pd, sp))
                C.check(L.st_grayscale(ctx, po, 84, ch, 0, pi, sp))
        el, ev, pl = timed(eng, run_steps, KS)
        r.update({"value": head.n_global * KS / el, "ms_per_step": el / KS * 1e3, "steps": KS,
                  "note": "value: env-steps/s of st_step + st_grayscale (obs_type=%r), eager launches"
                          % ("grayscale" if ch == 1 else "rgb")})
        out[name] = r
        del img
    return out


def clear_heavy(head, cfg_kw, C, ShardedTetris, timed, roofline, kname_of, dev, s, sp, rank, world,
                W, H, K, WU, aseed, config, launch):
    """Clear-heavy regime: uniform actions almost never clear a
    line, so the same st_step is also timed on an action stream that a greedy
    placement player (st_policy_greedy, 3% random) produced from the same start
    state: recorded untimed, then replayed from a snapshot of that start state
    through the same launch path."""
    n_global = head.n_global
    ce = ShardedTetris(n_global, seed=1000, rank=rank, world=world, device=dev,
                       autoreset="same_step", width=W, height=H, **cfg_kw).engine
    L = ce._L
    po, pr, pd = head.ptrs
    rew = head.sh._rew
    ce.reset()
    torch.cuda.synchronize(dev)
    snap = ce.save()
    gact = torch.empty((WU + K, ce.n), dtype=torch.uint8, device=dev)
    cleared = torch.zeros((), dtype=torch.int64, device=dev)
    with torch.cuda.stream(s):
        for t in range(WU + K):
            ce.policy_greedy(t, seed=aseed, explore=30, out=gact[t])
            C.check(L.st_step(ce._ctx, ctypes.c_void_p(gact[t].data_ptr()), po, pr, pd, sp))
            if t >= WU and config == "c3":  # default rewards: +100 per cleared line
                cleared += rew.clamp(min=0).sum()
    torch.cuda.synchronize(dev)
    n_cleared = int(cleared.item())
    ce.load(snap)
    gptr = [ctypes.c_void_p(gact[t].data_ptr()) for t in range(WU + K)]
    with torch.cuda.stream(s):
        for t in range(WU):
            C.check(L.st_step(ce._ctx, gptr[t], po, pr, pd, sp))
    torch.cuda.synchronize(dev)
    garr = (ctypes.c_void_p * (WU + K))(*[a.value for a in gptr])

    def run_eager():
        if launch == "native":  # the headline's launch path: one st_step_n call
            C.check(L.st_step_n(ce._ctx, ctypes.addressof(garr) + WU * ctypes.sizeof(ctypes.c_void_p), K, po, None,
                                pr, pd, sp))
            return
        for t in range(WU, WU + K):
            C.check(L.st_step(ce._ctx, gptr[t], po, pr, pd, sp))
    g = None
    if launch == "graph":
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            run_eager()
        torch.cuda.synchronize(dev)
    el, ev, pl = timed(ce, g.replay if g is not None else run_eager, K)
    kern_us = ev * 1e3 / K
    bpe = (182.0 + 184.0 * pl)
    r = {"value": n_global * K / el, "ms_per_step": el / K * 1e3, "p_lock": pl,
         "lines_per_env_step": (n_cleared / 100.0 / (ce.n * K)) if config == "c3" else None,
         "actions": "st_policy_greedy (greedy placement, 3% uniform), recorded then replayed",
         "roofline": roofline(kern_us, bpe, ce.n, kname_of("step", False, not cfg_kw), grid=None, extra=
                              {"bytes_formula": "SURVEY 8(d): 182 + 184 p_lock", "p_lock": pl,
                               "traffic_note": "same kernel and launch shape as the headline: a PMC pass "
                                               "cannot tell the two workloads apart"})}
    del g
    ce.close()
    return r


if __name__ == "__main__":
    main()
