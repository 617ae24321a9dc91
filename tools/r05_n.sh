#!/bin/bash
# Round 5: state-store cache policy A/B (board / counter rows / MT words
# write-back instead of nt; outputs stay nt).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05n
B=$R/gym-simpletetris_amd/csrc/build
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_st0.so $B/lib_st1.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05n/ab_state_cpol.txt || exit 1
  done
done
