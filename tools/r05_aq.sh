#!/bin/bash
# Round 5: the driver's shape with the spawn counter as a device reduction
# (bench_prev.py) vs a pinned-host copy (bench.py), alternating.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05aq
for i in 1 2 3 4; do
  for b in bench_prev.py bench.py; do
    timeout -k 10 120 python $b --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r05aq/tmp.json 2>> gpurun_out/r05aq/err.txt || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/r05aq/tmp.json').read().strip().splitlines()[-1]); print('$b', d['value'], d['ms_per_step']*1e3, d['roofline']['event_us_per_launch'])" >> gpurun_out/r05aq/k20.txt || exit 1
  done
done
