#!/bin/bash
# Round 5: st_rollout's packed obs stores, cache policy: nt (current) vs
# write-back (lib_rowb) vs sc1 nt (lib_rosc) -- rollout only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05w
B=$R/gym-simpletetris_amd/csrc/build
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_rowb.so $B/lib_rosc.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05w/ab.txt || exit 1
  done
done
