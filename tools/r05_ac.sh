#!/bin/bash
# Round 5: the harness's rollout with the engine's action check mode as the
# bench has it ('async': the kernel's sticky flag in mapped host memory).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ac
for i in 1 2; do
  for va in True async False; do
    echo "validate=$va $(AB_VALIDATE=$va timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05ac/ro.txt || exit 1
  done
done
