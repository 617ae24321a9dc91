#!/bin/bash
# Bench-only A/B over several builds of libsimpletetris.so (two alternating rounds).
# usage: [WARMUP=W] [STEPS=K] tools/ab_libs.sh lib1.so lib2.so ...
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for round in 1 2; do
  for lib in "$@"; do
    ST_LIB="$lib" timeout -k 10 200 python bench.py --steps ${STEPS:-500} --warmup ${WARMUP:-50} --no-cpu-baseline \
     | python -c "import json,sys; d=json.load(sys.stdin); v=d['variants']; print('$(basename $lib): step=%.3f step_f32=%.3f rollout_packed=%.3f rollout_f32=%.3f us/step' % (d['ms_per_step']*1e3, v['step_f32']['ms_per_step']*1e3, v['rollout_packed']['ms_per_step']*1e3, v['rollout_f32']['ms_per_step']*1e3))" || exit 1
  done
done
