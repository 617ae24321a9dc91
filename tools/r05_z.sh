#!/bin/bash
# Round 5: why the bench's rollout (1.34 us/step) is slower than the A/B
# harness's (1.22-1.24): the harness cold, then the full bench, then the
# harness again right after it, and with 40 rollout launches.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05z
O=gpurun_out/r05z
echo "cold $(timeout -k 10 120 python tools/ab_step.py 1000)" >> $O/ro.txt || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
echo "after-bench $(timeout -k 10 120 python tools/ab_step.py 1000)" >> $O/ro.txt || exit 1
echo "after-bench-k4000 $(timeout -k 10 120 python tools/ab_step.py 4000)" >> $O/ro.txt || exit 1
echo "bench-rollout-only $(timeout -k 10 300 python bench.py --no-cpu-baseline --no-surfaces --steps 1000 --warmup 100 | python -c "import json,sys; d=json.load(sys.stdin); print(d['variants']['rollout_packed']['ms_per_step']*1e3, d['variants']['rollout_packed']['roofline']['event_us_per_launch'])")" >> $O/ro.txt || exit 1
