#!/bin/bash
# Round 5: the harness rollout's p_lock beside the bench's (0.2117).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ae
echo "$(timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05ae/ro.txt || exit 1
echo "wu3000 $(AB_WU=3000 timeout -k 10 180 python tools/ab_step.py 1000)" >> gpurun_out/r05ae/ro.txt || exit 1
