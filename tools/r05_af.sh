#!/bin/bash
# Round 5: rollout timing vs what precedes the timed launches: nothing (the
# warm-up launch still running), a synchronize, a synchronize + 0.1 / 1 / 10
# ms idle, a synchronize + the p_lock read.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05af
for i in 1 2; do
  for pre in none sync sleep0.1 sleep1 sleep10 plock; do
    echo "pre=$pre $(AB_PRE=$pre timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05af/ro.txt || exit 1
  done
done
