#!/bin/bash
# A/B of rollout variants (build/lib_*.so named on the command line) against
# the tree's library, 65,536 and 32,768 envs, packed and float32, alternated.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-roqab}
N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
for n in 65536 32768; do
  for i in 1 2; do
    for lib in $N "$@"; do
      AB_N=$n ST_LIB=$lib AB_LABEL="$(basename $lib) n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 f32 || exit 1
    done
  done
done | tee gpurun_out/ab_$TAG.txt
