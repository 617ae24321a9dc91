#!/bin/bash
# Bench-only A/B of HIP runtime environment settings, alternating rounds.
# usage: tools/ab_env.sh "X=1" "HIP_FORCE_DEV_KERNARG=1" ...   (each arg: env assignments)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for round in 1 2 3; do
  for e in "$@"; do
    for shape in "20:5" "4000:100"; do
      k=${shape%%:*}; w=${shape##*:}
      env $e timeout -k 10 120 python bench.py --steps $k --warmup $w --no-extras --no-cpu-baseline \
       | python -c "import json,sys; d=json.load(sys.stdin); print('[%s] K=%s: %.3f us/step wall, %.3f event, %.3e env-steps/s' % ('$e', '$k', d['ms_per_step']*1e3, d['event_ms_per_step']*1e3, d['value']))" || exit 1
    done
  done
done
