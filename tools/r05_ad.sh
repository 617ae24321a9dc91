#!/bin/bash
# Round 5: the bench's rollout line before / after the float32 step variant
# (ST_BENCH_RO_FIRST=1 runs the rollout first), against the harness.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ad
O=gpurun_out/r05ad
for i in 1 2; do
  for rf in 0 1; do
    echo "ro_first=$rf $(ST_BENCH_RO_FIRST=$rf timeout -k 10 300 python bench.py --no-cpu-baseline --no-surfaces --steps 1000 --warmup 100 | python -c "import json,sys; d=json.load(sys.stdin); r=d['variants']['rollout_packed']; print(r['ms_per_step']*1e3, r['roofline']['event_us_per_launch'], r['p_lock'])")" >> $O/ro.txt || exit 1
  done
done
echo "harness $(timeout -k 10 120 python tools/ab_step.py 1000)" >> $O/ro.txt || exit 1
