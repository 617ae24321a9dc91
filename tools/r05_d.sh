#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05d
B=gym-simpletetris_amd/csrc/build
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
    >> gpurun_out/r05d/k20_repeat.jsonl 2>> gpurun_out/r05d/k20.err || exit 1
done
TAG=r05d_ab_ecount timeout -k 10 600 bash tools/ab.sh step 3 gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so $B/lib_ecount.so || exit 1
ST_LIB=$R/$B/lib_ldswin.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_long_horizon.py -k "rollout or soak" > gpurun_out/r05d/pytest_ldswin.log 2>&1 || exit 1
TAG=r05d_ab_ldswin timeout -k 10 300 bash tools/ab.sh rollout 3 gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so $B/lib_ldswin.so || exit 1
