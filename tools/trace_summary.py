"""Per-kernel duration distribution from a rocprofv3 kernel trace (csv).

usage: python tools/trace_summary.py <..._kernel_trace.csv> [min_run]
       python tools/trace_summary.py --json TAG [--rollout-k K] <trace.csv[:bench.json]>...
         -> JSON on stdout: per engine kernel@grid@kK (bench.launch_key; K =
            steps per launch: K for k_rollout, 1 otherwise), the longest
            run's traced duration stats and -- given the JSON line of the
            traced bench run after a colon -- that run's p_lock for the key,
            with bench.kernel_source_sha() of the sources
            (profiles/<TAG>_trace.json, read by bench.py's roofline)

bench.py launches the same kernel in several workloads (the headline's
warm-up and timed graph, the C2 batch with a smaller grid, the clear-heavy
replay), so the launches are grouped by (kernel, grid size) and split into
runs: maximal sequences of that key in launch order with no other kernel in
between.  Each run of >= min_run launches (default 50) is listed with its
mean and median (rocprofv3 --stats reports the mean of ALL launches of a
kernel name, i.e. of every workload mixed).
"""
import csv
import statistics
import sys


def short(name):
    return name.replace("st::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def split_runs(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs = []  # [key, [durations]]
    for r in rows:
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        key = (short(r["Kernel_Name"]), grid)
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if runs and runs[-1][0] == key:
            runs[-1][1].append(d)
        else:
            runs.append([key, [d]])
    return runs


def stats(v):
    s = sorted(v)
    q = lambda f: s[min(len(s) - 1, int(f * len(s)))] / 1e3  # noqa: E731
    return {"launches": len(v), "mean_us": statistics.mean(v) / 1e3,
            "median_us": statistics.median(v) / 1e3, "p10_us": q(0.1), "p90_us": q(0.9)}


def to_json(tag, paths):
    import json
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench
    from pmc_summary import bench_p_lock
    rollout_k = 100
    if "--rollout-k" in paths:
        i = paths.index("--rollout-k")
        rollout_k = int(paths[i + 1])
        paths = paths[:i] + paths[i + 2:]
    longest = {}
    for spec in paths:  # earlier files win ties
        path, _, bj = spec.partition(":")
        pl = bench_p_lock(bj)
        for key, v in split_runs(path):
            k = f"{key[0]}@{key[1]}@k{rollout_k if key[0].startswith('k_rollout') else 1}"
            if key[0].startswith("k_") and len(v) > longest.get(k, {}).get("launches", 0):
                longest[k] = dict(stats(v), trace=os.path.basename(path), p_lock=pl.get(k))
    print(json.dumps({"tag": tag, "kernel_source_sha": bench.kernel_source_sha(), "rollout_k": rollout_k,
                      "kernels": longest}, indent=1))


def main():
    if sys.argv[1] == "--json":
        return to_json(sys.argv[2], sys.argv[3:])
    path = sys.argv[1]
    min_run = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    runs = split_runs(path)
    print(f"{'run':>3s} {'kernel':42s} {'grid':>8s} {'calls':>6s} {'mean_us':>8s} {'median':>8s} "
          f"{'p10':>8s} {'p90':>8s}")
    for i, (key, v) in enumerate(runs):
        if len(v) < min_run:
            continue
        s = sorted(v)
        q = lambda f: s[min(len(s) - 1, int(f * len(s)))] / 1e3  # noqa: E731
        print(f"{i:3d} {key[0][:42]:42s} {key[1]:>8s} {len(v):6d} {statistics.mean(v) / 1e3:8.3f} "
              f"{statistics.median(v) / 1e3:8.3f} {q(0.1):8.3f} {q(0.9):8.3f}")


if __name__ == "__main__":
    main()
