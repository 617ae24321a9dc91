#!/bin/bash
# Rollout A/B: parity tests of the rollout path on the in-tree build, then
# tools/ab_rollout.py alternating baseline / new (packed + f32), 3 rounds,
# then the new build's rollout phase stamps.
# usage: tools/ab_ro.sh <baseline .so>
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-abro}
BASE="$1"; NEW="$R/gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "rollout or soak or interop" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_$TAG.log; grep -m3 "^E " gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for lib in "$BASE" "$NEW"; do
    ST_LIB="$lib" AB_LABEL=$(basename $lib) timeout -k 10 120 python tools/ab_rollout.py 100 20 f32 || exit 1
  done
done | tee gpurun_out/ab_ro_$TAG.txt
timeout -k 10 120 python tools/ro_stamps.py 100 6 | tee gpurun_out/ro_stamps_$TAG.txt
