#!/bin/bash
# Timing-only ablations of the three-wave st_rollout (results are NOT valid
# games), 65,536 envs, 100-step launches: 0 = none, 16 = no MT window reload,
# 32 = no next-generation chunk, 48 = neither, 2 = no draw at all.
# Needs: make -C gym-simpletetris_amd/csrc variant V=ablation DEFS=-DST_ABLATION=1
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
A=$R/gym-simpletetris_amd/csrc/build/lib_ablation.so
TAG=${TAG:-ro3}
for ab in 0 16 32 48 2 0 16 32 48 2; do
  ST_LIB=$A ST_ABLATE=$ab timeout -k 10 120 python tools/ab_rollout.py 100 20 || exit 1
done | tee gpurun_out/ro_ablate_$TAG.txt
