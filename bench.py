#!/usr/bin/env python
"""bench.py -- env-steps/s of the MI355X batched SimpleTetris engine.

Metric (BASELINE.json): env-steps/sec at 65,536 parallel 10x20 boards per GPU,
1 -> 8 GPU weak scaling.  One "step" = one batched TetrisEngine.step
(tetris_env.py:243-304) over every env of the job, fed by synthetic uniform
actions a[t, e] = splitmix64(seed ^ ((t << 32) ^ e)) % 7 that are generated
into HBM before the timed region.  Envs auto-reset inside the
step kernel when they die (reference driver `if done: env.reset()`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4] [--obs packed|f32] [--clear-heavy]

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
try:
    METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
except Exception:  # noqa: BLE001
    METRIC = "env-steps/sec at 65 536 parallel 10\u00d720 boards; 1\u21928 GPU scaling"

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
    amortised next MT generation (2 x 2,496 B read + 2,496 B written per
    ~476 draws) 15.7."""
    always = (1 + 4 + 4 + 4 * width) + (4 + 4 + 4 + 1 + 4 * width)
    if f32:
        always += 4 * width * height
    lock = 2 * 13 * 4 + 4 * width + 8 + 15.7
    return always + lock * p_lock


def rollout_bytes(width: int, height: int, p_lock: float, f32: bool, k: int) -> float:
    """Algorithmic HBM bytes per env-step of the K-step rollout kernel: per
    step read action 1, write packed obs 4W + reward 4 + done 1 (+ float32
    obs 4WH); per lock MT words 8 + amortised next generation 15.7; per launch the state
    (board 4W + 14 counters + piece) read and written once, / K."""
    step = 1 + 4 * width + 4 + 1 + (4 * width * height if f32 else 0)
    state = 2 * (4 * width + 15 * 4)
    return step + 23.7 * p_lock + state / k


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
    ap.add_argument("--steps", type=int, default=4000,
                    help="timed steps (default spans >= 2 MT generations of a typical env, ~1,650 steps each)")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--obs", choices=("packed", "f32"), default="packed")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    ap.add_argument("--gather", action="store_true", help="also time a per-step RCCL gather")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--rollout-chunk", type=int, default=100, help="steps per st_rollout launch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="timed region only (profiling)")
    ap.add_argument("--clear-heavy", action="store_true",
                    help="also time st_step on a greedy-player (line-clearing) action stream; off by "
                         "default so that the headline kernel's rocprofv3 average covers only the "
                         "headline workload")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    # ST_BENCH_SHARED_GPU=1 (tests only): every rank on cuda:0, to exercise the
    # N>1 logic on a one-GPU box with --backend gloo
    dev_idx = 0 if os.environ.get("ST_BENCH_SHARED_GPU") == "1" else local_rank
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

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

    def spawned():
        st = eng.state_tensors(("stats",), sync=False)["stats"][6:13, :n_local]
        return int(st.to(torch.int64).sum().item())

    def timed(run, nsteps):
        """Run `run()` (enqueues exactly nsteps steps on s) inside the timed
        region: barrier + synchronize on both sides, max over ranks."""
        c0 = spawned()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            ev0.record(s)
            run()
            ev1.record(s)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        # every lock spawns exactly one piece (the new piece, or the auto-reset's)
        p_lock = (spawned() - c0) / float(n_local * nsteps)
        return elapsed, ev0.elapsed_time(ev1), p_lock

    class _Eager:  # --no-graph (PMC passes): the same launches, eagerly
        def __init__(self, use_f32):
            self.f = use_f32

        def replay(self):
            for t in range(WU, WU + K):
                if self.f:
                    C.check(L.st_step_f32(ctx, act_ptrs[t], p_obs, p_f32, p_rew, p_done, sp))
                else:
                    C.check(L.st_step(ctx, act_ptrs[t], p_obs, p_rew, p_done, sp))

    def step_graph(use_f32):
        if args.no_graph:
            return _Eager(use_f32)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for t in range(WU, WU + K):
                if use_f32:
                    C.check(L.st_step_f32(ctx, act_ptrs[t], p_obs, p_f32, p_rew, p_done, sp))
                else:
                    C.check(L.st_step(ctx, act_ptrs[t], p_obs, p_rew, p_done, sp))
        torch.cuda.synchronize(dev)
        return g

    def roofline(kern_ms, bpe, launch_steps, kname):
        achieved = bpe * n_local * launch_steps / (kern_ms * 1e-3) / 1e9
        traffic, pmc_file = load_pmc(kname)
        return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                "kernel_us": kern_ms * 1e3, "bytes_per_env_step": bpe,
                "bytes_per_launch": bpe * n_local * launch_steps, "traffic_source": pmc_file}

    # ---------------- headline: K single steps (st_step), graph-replayed ----------------
    graph = step_graph(f32)

    def run_main():
        graph.replay()
    elapsed, ev_ms, p_lock = timed(run_main, K)
    value = n_global * K / elapsed
    event_ms = ev_ms / K
    sc0 = not cfg_kw  # no scoring flags: the SC0 specialization (st_kernels.hip launch_step)

    def kname_of(kind, use_f32):  # rocprofv3's demangled name of the 10x20 kernel
        b = lambda v: "true" if v else "false"  # noqa: E731
        if kind == "step":
            return f"k_step<10, 20, {b(use_f32)}, false, {b(sc0)}>"
        return f"k_rollout<10, 20, {b(use_f32)}, {b(sc0)}>"
    kname = kname_of("step", f32)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": WU,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (uniform splitmix64 actions, seeds 1000 + global env index)",
        "config": {
            "workload": f"{'C4' if args.config == 'c4' else 'C3'}: {n_local} parallel {W}x{H} boards "
                        f"per GPU, one st_step per step, ram obs ({args.obs}), auto-reset, "
                        + ("advanced_clears+penalise_holes_increase+penalise_height_increase"
                           if args.config == "c4" else "default rewards"),
            "envs_per_gpu": n_local,
            "envs_total": n_global,
            "board": f"{W}x{H}",
            "obs": args.obs,
            "launch": "eager" if args.no_graph else "hipGraph of K st_step launches",
            "parallelism": f"env-shard x{world}",
        },
        "p_lock": p_lock,
        "event_ms_per_step": event_ms,
        # graph launches run back to back (rocprofv3: ~0 gap), so the event
        # time of the timed region / K is the kernel's average duration
        "roofline": roofline(event_ms, algorithmic_bytes(W, H, p_lock, f32), 1, kname),
    }
    del graph

    if not args.no_extras:
        variants = {}
        if not f32:  # the same st_step with the reference's float32 obs fused in
            if obs_f32 is None:  # keep the tensor alive while graphs/launches use it
                obs_f32 = torch.zeros((n_local, W, H), dtype=torch.float32, device=dev)
                p_f32 = ctypes.c_void_p(obs_f32.data_ptr())
            g = step_graph(True)
            el, ev, pl = timed(g.replay, K)
            variants["step_f32"] = {
                "value": n_global * K / el, "ms_per_step": el / K * 1e3, "p_lock": pl,
                "roofline": roofline(ev / K, algorithmic_bytes(W, H, pl, True), 1,
                                     kname_of("step", True))}
            del g
        # K-step rollout kernel (st_rollout): CH steps per launch
        CH = min(args.rollout_chunk, K)
        nch = K // CH
        ro = torch.empty((CH, W, n_local), dtype=torch.int32, device=dev)
        rr = torch.empty((CH, n_local), dtype=torch.int32, device=dev)
        rd = torch.empty((CH, n_local), dtype=torch.uint8, device=dev)
        for use_f32 in (False, True):
            rf = torch.empty((CH, n_local, W, H), dtype=torch.float32, device=dev) if use_f32 else None
            aptr = [ctypes.c_void_p(actions[WU + c * CH].data_ptr()) for c in range(nch)]
            ptrs = [ctypes.c_void_p(x.data_ptr()) if x is not None else None for x in (ro, rf, rr, rd)]

            def run_ro():
                for c in range(nch):
                    C.check(L.st_rollout(ctx, CH, aptr[c], *ptrs, sp))
            with torch.cuda.stream(s):  # warm-up launch
                C.check(L.st_rollout(ctx, CH, aptr[0], *ptrs, sp))
            el, ev, pl = timed(run_ro, nch * CH)
            key = "rollout_f32" if use_f32 else "rollout_packed"
            variants[key] = {
                "value": n_global * nch * CH / el, "ms_per_step": el / (nch * CH) * 1e3,
                "steps_per_launch": CH, "p_lock": pl,
                "roofline": roofline(ev / nch, rollout_bytes(W, H, pl, use_f32, CH), CH,
                                     kname_of("rollout", use_f32))}
            del rf

        def clear_heavy(variants):
            # Clear-heavy regime: uniform actions almost never clear
            # a line, so the same st_step is also timed on an action stream that
            # a greedy placement player (st_policy_greedy, 3% random) produced from
            # the same start state: recorded untimed, then replayed from a
            # snapshot of that start state through the same hipGraph path.
            ce = ShardedTetris(n_global, seed=1000, rank=rank, world=world, device=dev,
                               autoreset="same_step", width=W, height=H, **cfg_kw).engine
            ce.reset()
            snap = ce.save()
            gact = torch.empty((WU + K, n_local), dtype=torch.uint8, device=dev)
            cleared = torch.zeros((), dtype=torch.int64, device=dev)
            with torch.cuda.stream(s):
                for t in range(WU + K):
                    ce.policy_greedy(t, seed=aseed, explore=30, out=gact[t])
                    C.check(L.st_step(ce._ctx, ctypes.c_void_p(gact[t].data_ptr()), p_obs, p_rew, p_done, sp))
                    if t >= WU:  # default rewards: +100 per cleared line
                        cleared += rew_v.clamp(min=0).sum()
            torch.cuda.synchronize(dev)
            n_cleared = int(cleared.item())
            ce.load(snap)
            del snap
            gptr = [ctypes.c_void_p(gact[t].data_ptr()) for t in range(WU + K)]
            with torch.cuda.stream(s):
                for t in range(WU):
                    C.check(L.st_step(ce._ctx, gptr[t], p_obs, p_rew, p_done, sp))
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for t in range(WU, WU + K):
                    C.check(L.st_step(ce._ctx, gptr[t], p_obs, p_rew, p_done, sp))
            torch.cuda.synchronize(dev)
            el, ev, _ = timed(g.replay, K)
            variants["step_clear_heavy"] = {
                "value": n_global * K / el, "ms_per_step": el / K * 1e3,
                "lines_per_env_step": (n_cleared / 100.0 / (n_local * K)) if args.config == "c3" else None,
                "actions": "st_policy_greedy (greedy placement, 3% uniform), recorded then replayed",
                "kernel_us": ev / K * 1e3}
            del g, ce

        if args.clear_heavy:
            clear_heavy(variants)
        out["variants"] = variants
        if args.gather and world > 1:
            torch.cuda.synchronize(dev)
            dist.barrier()
            g0 = time.perf_counter()
            G = min(K, 200)
            for i in range(G):
                with torch.cuda.stream(s):
                    step(WU + i, sp)
                s.synchronize()
                sh.gather(cpu=args.backend != "nccl")
            torch.cuda.synchronize(dev)
            dist.barrier()
            gdt = time.perf_counter() - g0
            tt = torch.tensor([gdt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            gdt = float(tt.item())
            out["gather_variant"] = {"value": n_global * G / gdt, "ms_per_step": gdt / G * 1e3,
                                     "steps": G, "bytes_per_rank_per_step": sh.buf.numel() * 4,
                                     "note": "eager st_step + RCCL gather of packed obs/reward/done to rank 0"}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, cfg_kw)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
