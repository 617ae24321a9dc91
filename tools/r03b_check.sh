#!/bin/bash
# Full GPU suite, then st_step and st_rollout A/B against build/lib_base.so
# (the round-start kernels) and the rollout stamps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-r03b}
B=gym-simpletetris_amd/csrc/build; N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$TAG.log; grep -m5 "^E " gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
TAG=$TAG bash tools/ab_step_libs.sh 3 $B/lib_base.so $N || exit 1
for n in 65536 32768; do
  for i in 1 2; do
    for lib in $B/lib_base.so $N; do
      AB_N=$n ST_LIB=$lib AB_LABEL="$(basename $lib) n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 f32 || exit 1
    done
  done
done | tee gpurun_out/ab_ro_$TAG.txt
timeout -k 10 120 python tools/ro_stamps.py 100 6 | tee gpurun_out/stamps_$TAG.txt
