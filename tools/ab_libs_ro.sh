#!/bin/bash
# Rollout timing (tools/ab_rollout.py, packed, 65,536 envs) of several
# library builds, alternated over rounds.  usage: tools/ab_libs_ro.sh R lib...
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-abl}
ROUNDS=$1; shift
for i in $(seq $ROUNDS); do
  for lib in "$@"; do
    ST_LIB="$lib" AB_LABEL=$(basename $lib) timeout -k 10 120 python tools/ab_rollout.py 100 10 ${AB_F32:+f32} || exit 1
  done
done | tee gpurun_out/ab_libs_ro_$TAG.txt
