#!/bin/bash
# The driver's bench command as the FIRST command of a fresh gpurun lease
# (VERDICT r4 #2), then the same shape repeated on the now-warm box, headline
# only.  Every run carries debug.region_probe (bench.py: the region's host
# submission timeline and per-launch event spans).
# Usage (from gpurun): bash tools/fresh_lease.sh TAG
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
TAG="${1:-r05}"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/fresh_driver.json" 2> "$O/fresh_driver.err" || exit 1
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
    >> "$O/k20_repeat.jsonl" 2>> "$O/k20_repeat.err" || exit 1
done
timeout -k 10 120 python bench.py --steps 4000 --warmup 100 --no-extras --no-cpu-baseline \
  > "$O/k4000.json" 2>> "$O/k4000.err" || exit 1
