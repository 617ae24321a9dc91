#!/bin/bash
# Round 5, call b: first-launch host cost probe (kernarg modes), early-counter
# A/B + its parity, split of the counter-store ablation.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05b
B=gym-simpletetris_amd/csrc/build
timeout -k 10 120 python tools/first_launch_probe.py > gpurun_out/r05b/first_launch_kernarg1.jsonl || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python tools/first_launch_probe.py > gpurun_out/r05b/first_launch_kernarg0.jsonl || exit 1
ST_LIB=$R/$B/lib_ecnt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_long_horizon.py -k "st_step or c2_shape" > gpurun_out/r05b/pytest_ecnt.log 2>&1 || exit 1
TAG=r05b_ab_ecnt timeout -k 10 600 bash tools/ab.sh step 3 gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so $B/lib_ecnt.so || exit 1
ST_LIB=$R/$B/lib_ablation.so AB_BITS="0 16384 32768 2048 0" TAG=r05b_split EXTRA="--steps 2000 --warmup 100" \
  timeout -k 10 300 bash tools/ablate.sh || exit 1
