#!/bin/bash
# Round 5: the in-process rollout probe with a synchronize between its
# warm-up launch and the timed launches (as timed() has).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ap
for sy in 0 1; do
  ST_BENCH_RO_PROBE=1 ST_BENCH_RO_PROBE_SYNC=$sy timeout -k 10 300 python bench.py --no-cpu-baseline --no-surfaces --steps 1000 --warmup 100 > gpurun_out/r05ap/b$sy.json 2> gpurun_out/r05ap/b$sy.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r05ap/b$sy.json').read().strip().splitlines()[-1]); r=d['variants']['rollout_packed']; print('sync=$sy bench line', r['ms_per_step']*1e3)" >> gpurun_out/r05ap/ro.txt || exit 1
  grep ro_probe gpurun_out/r05ap/b$sy.err >> gpurun_out/r05ap/ro.txt || exit 1
done
