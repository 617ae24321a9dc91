#!/bin/bash
# Round 5: the rollout after the p_lock read (stats copy + torch reduction):
# its first use in the process vs a warmed one.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ah
for i in 1 2; do
  for pre in none copy torchsum alloc plock; do
    echo "pre=$pre $(AB_PRE=$pre timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05ah/ro.txt || exit 1
  done
done
