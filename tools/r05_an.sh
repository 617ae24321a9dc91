#!/bin/bash
# Round 5: inside bench.py's process, its rollout line beside the same
# engine's launches timed harness-style (ST_BENCH_RO_PROBE=1).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05an
for i in 1 2; do
  ST_BENCH_RO_PROBE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-surfaces --steps 1000 --warmup 100 > gpurun_out/r05an/b$i.json 2> gpurun_out/r05an/b$i.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r05an/b$i.json').read().strip().splitlines()[-1]); r=d['variants']['rollout_packed']; print('bench line', r['ms_per_step']*1e3, r['roofline']['event_us_per_launch'])" >> gpurun_out/r05an/ro.txt || exit 1
  grep ro_probe gpurun_out/r05an/b$i.err >> gpurun_out/r05an/ro.txt || exit 1
done
