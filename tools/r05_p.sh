#!/bin/bash
# Round 5: the rollout output wave's phases (finer stamps), and the chunk
# lag A/B (ST_RO_CHLAG=1) with its rollout parity tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05p
B=$R/gym-simpletetris_amd/csrc/build
timeout -k 10 150 python tools/ro_stamps.py > gpurun_out/r05p/ro_stamps_cur.txt 2>&1 || exit 1
ST_LIB=$B/lib_chlag.so timeout -k 10 150 python tools/ro_stamps.py > gpurun_out/r05p/ro_stamps_chlag.txt 2>&1 || exit 1
ST_LIB=$B/lib_chlagep.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py -m gpu -x -q -k "rollout or soak or long" --timeout 300 --timeout-method thread > gpurun_out/r05p/pytest_chlag.log 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_chlag.so $B/lib_chlagep.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05p/ab_chlag.txt || exit 1
  done
done
TAG=r05 timeout -k 10 900 bash tools/nsweep.sh > /dev/null || exit 1
