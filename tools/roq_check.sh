#!/bin/bash
# Queued-draw st_rollout: the rollout parity tests, then an A/B against the
# previous kernel (build/lib_base.so) at 65,536 / 32,768 envs and the phase
# stamps of the new kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-roq}
B=gym-simpletetris_amd/csrc/build; N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "rollout or rejection or generation or rewind" > gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t_$TAG.log; grep -m5 "^E " gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_long_horizon.py \
  -k "st_rollout or soak" >> gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t_$TAG.log; grep -m5 "^E " gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit $rc
for n in 65536 32768; do
  for i in 1 2; do
    for lib in $B/lib_base.so $N; do
      AB_N=$n ST_LIB=$lib AB_LABEL="$(basename $lib) n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 f32 || exit 1
    done
  done
done | tee gpurun_out/ab_vs_base_$TAG.txt
timeout -k 10 120 python tools/ro_stamps.py 100 6 | tee gpurun_out/stamps_$TAG.txt
