#!/bin/bash
# A/B of two builds of libsimpletetris.so: GPU parity tests on the new build,
# then stamp phase split + bench (step variants) for each library, alternated.
# usage: tools/ab_lib.sh <baseline .so>   (new = the in-tree library)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-ab}
BASE="$1"; NEW="$R/gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so"
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_$TAG.log; grep -m3 "^E " gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for lib in "$BASE" "$NEW"; do
  echo "== $(basename $lib)"
  ST_LIB="$lib" timeout -k 10 200 python tools/stamps.py || exit 1
done
for lib in "$BASE" "$NEW" "$BASE" "$NEW"; do
  ST_LIB="$lib" timeout -k 10 200 python bench.py --steps 500 --warmup 50 --no-cpu-baseline \
   | python -c "import json,sys; d=json.load(sys.stdin); v=d['variants']; print('$(basename $lib): step=%.3f step_f32=%.3f rollout_packed=%.3f rollout_f32=%.3f us/step' % (d['ms_per_step']*1e3, v['step_f32']['ms_per_step']*1e3, v['rollout_packed']['ms_per_step']*1e3, v['rollout_f32']['ms_per_step']*1e3))" || exit 1
done
