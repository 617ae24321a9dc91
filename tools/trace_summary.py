"""Per-kernel duration distribution from a rocprofv3 kernel trace (csv).

usage: python tools/trace_summary.py <..._kernel_trace.csv> [min_run]

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


def main():
    path = sys.argv[1]
    min_run = int(sys.argv[2]) if len(sys.argv) > 2 else 50
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
