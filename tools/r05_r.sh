#!/bin/bash
# Round 5: the rollout output wave's chunk at the start of each step
# (ST_RO_CHFIRST=1: its operand loads issued before that step's stores) --
# rollout parity, stamps, A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05r
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_chf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py -m gpu -x -q -k "rollout or soak or long" --timeout 300 --timeout-method thread > gpurun_out/r05r/pytest_chf.log 2>&1 || exit 1
ST_LIB=$B/lib_chf.so timeout -k 10 150 python tools/ro_stamps.py > gpurun_out/r05r/ro_stamps_chf.txt 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_chf.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05r/ab_chf.txt || exit 1
  done
done
