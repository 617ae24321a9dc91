#!/bin/bash
# Round 5: the rollout's chunk cadence change in the aged (steady) state --
# 3,000 st_steps before the timed rollouts (every env past its first MT
# generation) -- against the build before it (lib_pre, commit 31757e7).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05aa
B=$R/gym-simpletetris_amd/csrc/build
for i in 1 2 3; do
  for lib in $B/lib_pre.so $B/lib_cur.so; do
    echo "wu3000 $(AB_WU=3000 ST_LIB=$lib timeout -k 10 180 python tools/ab_step.py 1000)" >> gpurun_out/r05aa/ab.txt || exit 1
  done
done
for lib in $B/lib_pre.so $B/lib_cur.so; do
  echo "wu300 $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05aa/ab.txt || exit 1
done
