#!/bin/bash
# BASELINE configs C2 (4,096 boards) and C4 (reward-heavy flags) on one GPU.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.json && \
timeout -k 10 300 python bench.py --n-envs 4096 --no-cpu-baseline > gpurun_out/bench_c2.json && \
python - <<'PY'
import json
for f in ("gpurun_out/bench_c4.json", "gpurun_out/bench_c2.json"):
    d = json.load(open(f))
    print(f, d["config"]["workload"])
    print("  step  %.3e env-steps/s  %.3f us/step  frac %.3f" % (d["value"], d["ms_per_step"] * 1e3, d["roofline"]["frac"]))
    for k, v in d["variants"].items():
        print("  %-15s %.3e env-steps/s  %.3f us/step  frac %.3f" % (k, v["value"], v["ms_per_step"] * 1e3, v["roofline"]["frac"]))
PY
