#!/bin/bash
# The driver's bench shape (--steps 20 --warmup 5, headline only), alternated
# over env knobs (A/B).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for i in 1 2 3; do
  for va in async false; do
    ST_BENCH_VALIDATE=$va ST_BENCH_DEBUG=1 timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 5 2> gpurun_out/k20b_err.txt \
      | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('validate=$va wall_us=%.3f event_us=%.3f steady_us=%.3f value=%.4g' % (d['ms_per_step']*1e3, r['event_us_per_launch'], r['steady']['event_us_per_launch'], d['value']))" || exit 1
    grep -m1 timed gpurun_out/k20b_err.txt
  done
done | tee gpurun_out/k20_bench.txt
timeout -k 10 120 python tools/k20_first.py
