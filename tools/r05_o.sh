#!/bin/bash
# Round 5: st_rollout timing ablations (ablation build; results are not
# valid games): which wave's work sets the three-wave rollout's step.
# 1 no lock path, 2 no draw consumption, 8 no obs stores, 16 no MT chunks,
# 64 no reward/done stores, 160 logic skips the draw-queue wait, 288 logic
# skips the planes wait.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05o
export ST_LIB=$R/gym-simpletetris_amd/csrc/build/lib_ablation.so
for ab in 0 1 2 8 16 64 160 288 24 0; do
  echo "ablate=$ab $(ST_ABLATE=$ab timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05o/ro_ablate.txt || exit 1
done
