#!/bin/bash
# Round 5: the bench's spawn counter as a pinned-host copy (no torch kernel
# next to the timed region): the rollout line beside the harness-style probe,
# and the driver's shape.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ao
for i in 1 2; do
  ST_BENCH_RO_PROBE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-surfaces --steps 1000 --warmup 100 > gpurun_out/r05ao/b$i.json 2> gpurun_out/r05ao/b$i.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r05ao/b$i.json').read().strip().splitlines()[-1]); r=d['variants']['rollout_packed']; print('bench line', r['ms_per_step']*1e3, r['roofline']['event_us_per_launch'], r['p_lock'], 'head', d['value'], d['p_lock'])" >> gpurun_out/r05ao/ro.txt || exit 1
  grep ro_probe gpurun_out/r05ao/b$i.err >> gpurun_out/r05ao/ro.txt || exit 1
done
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline >> gpurun_out/r05ao/k20.jsonl 2>> gpurun_out/r05ao/k20.err || exit 1
done
