#!/bin/bash
# Round 5: store cache policy A/B (nt vs sc1 write-through vs sc1 + nt), then
# the GPU suite + smoke + bench lines of the SoA tree (TAG=r05a).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05m
B=$R/gym-simpletetris_amd/csrc/build
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_sc1.so $B/lib_sc1nt.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05m/ab_cpol.txt || exit 1
  done
done
TAG=r05a bash tools/gpu_final.sh
