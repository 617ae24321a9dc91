"""Per-kernel duration distribution from a rocprofv3 kernel trace (csv).

usage: python tools/trace_summary.py <..._kernel_trace.csv> [skip_first_n_per_kernel]

rocprofv3 --stats reports the MEAN duration; under the profiler the bench's
graph-replayed launches no longer run back to back (the tracer adds gaps) and
the mean picks up a slow tail, so the median is listed beside it.
"""
import collections
import csv
import statistics
import sys

skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("st::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    d[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(f"{'kernel':45s} {'calls':>6s} {'mean_us':>8s} {'median':>8s} {'p10':>8s} {'p90':>8s}")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = v[skip:] if len(v) > skip else v
    s = sorted(v)
    q = lambda f: s[min(len(s) - 1, int(f * len(s)))] / 1e3  # noqa: E731
    print(f"{k[:45]:45s} {len(v):6d} {statistics.mean(v) / 1e3:8.3f} {statistics.median(v) / 1e3:8.3f} {q(0.1):8.3f} {q(0.9):8.3f}")
