#!/usr/bin/env python
"""bench.py -- env-steps/s of the MI355X batched SimpleTetris engine.

Metric (BASELINE.json): env-steps/sec at 65,536 parallel 10x20 boards per GPU,
1 -> 8 GPU weak scaling.  One "step" = one batched TetrisEngine.step
(tetris_env.py:243-304) over every env of the job, fed by synthetic uniform
actions a[t, e] = splitmix64(seed ^ ((t << 32) ^ e)) % 7 that are generated
into HBM before the timed region.  Envs auto-reset inside the
step kernel when they die (reference driver `if done: env.reset()`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4] [--obs packed|f32]

N > 1 is launched by torch.distributed.run (one process per GPU, RCCL); each
rank owns a contiguous block of global env indices and no collective runs in
the timed steps ("scaling": "weak").  --gather additionally times one RCCL
gather of every shard's packed obs/reward/done to rank 0 per step.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-simpletetris_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    # BASELINE.json configs[2] / [3]
    "c3": dict(),
    "c4": dict(advanced_clears=True, penalise_holes_increase=True, penalise_height_increase=True),
}


def algorithmic_bytes(width: int, height: int, p_lock: float, f32: bool) -> float:
    """Algorithmic HBM bytes per env-step of the step kernel.
    Always: read action 1 + piece 4 + time 4 + board 4W; write piece 4 +
    time 4 + reward 4 + done 1 + packed obs 4W (+ float32 obs 4WH).
    Per lock: counters (score, lines, holes, piece_height, deaths, 7 counts,
    MT index) read + written 2*13*4, board write 4W, MT words read 8, and the
    amortised MT twist (2 x 2,496 B per 476 draws) 10.5."""
    always = (1 + 4 + 4 + 4 * width) + (4 + 4 + 4 + 1 + 4 * width)
    if f32:
        always += 4 * width * height
    lock = 2 * 13 * 4 + 4 * width + 8 + 10.5
    return always + lock * p_lock


def cpu_baseline(seconds: float, cfg_kw: dict):
    """Oracle (C restatement of the reference step, 1 core) on a bounded sample
    of the same workload: 4,096 envs, same seeds/actions, auto-reset."""
    from oracle import oracle as O
    n = 4096
    ob = O.OracleBatch(n, [1000 + e for e in range(n)], width=10, height=20, **cfg_kw)
    ob.reset()
    chunk = 64
    t_steps = 0
    t0 = time.perf_counter()
    while True:
        acts = O.splitmix64_actions(0x5EED, t_steps, chunk, n)
        ob.rollout(acts, want_obs=True, want_stats=False)
        t_steps += chunk
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return dict(value=n * t_steps / dt, unit="env-steps/s", cores=1, kind="port",
                sample=f"C oracle (oracle/tetris_oracle.c), {n} envs x {t_steps} steps, "
                       f"{dt:.1f} s on 1 host core, packed obs, auto-reset")


def load_pmc(kernel_prefix: str):
    """Per-launch HBM traffic from the newest committed PMC summary, if any
    (profiles/*_pmc.json written by tools/pmc_summary.py)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        for k, v in d.get("kernels", {}).items():
            if kernel_prefix in k:
                return v.get("hbm_bytes_per_launch"), os.path.basename(f)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--obs", choices=("packed", "f32"), default="packed")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    ap.add_argument("--gather", action="store_true", help="also time a per-step RCCL gather")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="timed region only (profiling)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from gym_simpletetris_amd.distributed import ShardedTetris

    n_local = args.n_envs
    n_global = n_local * world
    cfg_kw = CONFIGS[args.config]
    W, H = 10, 20
    K, WU = args.steps, args.warmup
    aseed = 0x5EED
    sh = ShardedTetris(n_global, seed=1000, rank=rank, world=world, device=dev,
                       autoreset="same_step", width=W, height=H, **cfg_kw)
    eng = sh.engine
    f32 = args.obs == "f32"
    obs_f32 = torch.zeros((n_local, W, H), dtype=torch.float32, device=dev) if f32 else None
    L = eng._L
    from gym_simpletetris_amd import _lib as C

    # inputs resident in HBM before timing
    actions = torch.empty((WU + K, n_local), dtype=torch.uint8, device=dev)
    for t in range(WU + K):
        eng.gen_actions(t, aseed, global_offset=sh.offset, out=actions[t])
    eng.reset()
    obs_v, rew_v, done_v = buffer = (sh._obs, sh._rew, sh._done)
    ctx = eng._ctx
    p_obs, p_rew, p_done = (ctypes.c_void_p(x.data_ptr()) for x in buffer)
    p_f32 = ctypes.c_void_p(obs_f32.data_ptr()) if f32 else None
    act_ptrs = [ctypes.c_void_p(actions[t].data_ptr()) for t in range(WU + K)]

    def step(t, stream):
        if f32:
            C.check(L.st_step_f32(ctx, act_ptrs[t], p_obs, p_f32, p_rew, p_done, stream))
        else:
            C.check(L.st_step(ctx, act_ptrs[t], p_obs, p_rew, p_done, stream))

    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    with torch.cuda.stream(s):
        for t in range(WU):
            step(t, sp)
    torch.cuda.synchronize(dev)

    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for t in range(WU, WU + K):
                step(t, sp)
        torch.cuda.synchronize(dev)

    def spawned():
        st = eng.state_tensors(("stats",))["stats"][6:13, :n_local]
        return int(st.to(torch.int64).sum().item())

    c0 = spawned()
    # ---------------- timed region: exactly K steps ----------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        ev0.record(s)
        if graph is not None:
            graph.replay()
        else:
            for t in range(WU, WU + K):
                step(t, sp)
        ev1.record(s)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # ---------------------------------------------------------------
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    c1 = spawned()
    # every lock spawns exactly one piece (new piece, or the auto-reset's)
    p_lock = (c1 - c0) / float(n_local * K)
    value = n_global * K / elapsed
    ms_per_step = elapsed / K * 1e3
    event_ms = ev0.elapsed_time(ev1) / K

    out = {
        "metric": "env-steps/sec at 65 536 parallel 10x20 boards per GPU (1->8 GPU weak scaling)",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": WU,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (uniform splitmix64 actions, seeds 1000 + global env index)",
        "config": {
            "workload": f"{'C4' if args.config == 'c4' else 'C3'}: {n_local} parallel {W}x{H} boards "
                        f"per GPU, ram obs ({args.obs}), auto-reset, "
                        + ("advanced_clears+penalise_holes_increase+penalise_height_increase"
                           if args.config == "c4" else "default rewards"),
            "envs_per_gpu": n_local,
            "envs_total": n_global,
            "board": f"{W}x{H}",
            "obs": args.obs,
            "launch": "hipGraph of K steps" if graph is not None else "eager",
            "parallelism": f"env-shard x{world}",
        },
        "p_lock": p_lock,
        "event_ms_per_step": event_ms,
    }

    # roofline of the step kernel.  In the hipGraph the K launches run back to
    # back (rocprofv3 shows ~0 gap), so the HIP-event time of the timed region
    # / K is the kernel's average launch duration.
    kern_ms = event_ms if graph is not None else None
    if kern_ms is None:  # eager: bracket R single launches with events
        R = min(K, 200)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(R)]
        with torch.cuda.stream(s):
            for i in range(R):
                evs[i][0].record(s)
                step(WU + i, sp)
                evs[i][1].record(s)
        torch.cuda.synchronize(dev)
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    bpe = algorithmic_bytes(W, H, p_lock, f32)
    achieved = bpe * n_local / (kern_ms * 1e-3) / 1e9
    kname = f"k_step<10, 20, {'true' if f32 else 'false'}>"
    traffic, pmc_file = load_pmc(kname)
    out["roofline"] = {
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
        "kernel": kname, "kernel_us": kern_ms * 1e3, "bytes_per_env_step": bpe,
        "bytes_per_launch": bpe * n_local, "traffic_source": pmc_file,
    }
    if not args.no_extras:
        if args.gather and world > 1:
            bufs_t = []
            torch.cuda.synchronize(dev)
            dist.barrier()
            g0 = time.perf_counter()
            G = min(K, 200)
            for i in range(G):
                with torch.cuda.stream(s):
                    step(WU + i, sp)
                s.synchronize()
                sh.gather()
            torch.cuda.synchronize(dev)
            dist.barrier()
            gdt = time.perf_counter() - g0
            tt = torch.tensor([gdt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            gdt = float(tt.item())
            out["gather_variant"] = {"value": n_global * G / gdt, "ms_per_step": gdt / G * 1e3,
                                     "steps": G, "bytes_per_rank_per_step": sh.buf.numel() * 4,
                                     "note": "eager step + RCCL gather of packed obs/reward/done to rank 0"}
            del bufs_t
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, cfg_kw)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
