#!/bin/bash
# st_step A/B of several library builds on one box: bench.py --no-extras
# (eager launches, 65,536 envs, C3) at K = 2000 and at the driver's K = 20,
# alternated over rounds.  usage: tools/ab_step_libs.sh ROUNDS lib...
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-abs}
ROUNDS=$1; shift
for i in $(seq $ROUNDS); do
  for lib in "$@"; do
    for K in 2000 20; do
      W=100; [ $K -eq 20 ] && W=5
      ST_LIB="$lib" timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --steps $K --warmup $W \
        | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('%-16s K=%-5d ms_per_step_us=%.3f event_us=%.3f steady_us=%.3f value=%.4g' % ('$(basename $lib)', $K, d['ms_per_step']*1e3, r['event_us_per_launch'], r['steady']['event_us_per_launch'], d['value']))" || exit 1
    done
  done
done | tee gpurun_out/ab_step_$TAG.txt
