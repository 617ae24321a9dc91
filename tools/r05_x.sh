#!/bin/bash
# Round 5: st_rollout's output wave building one next-generation chunk per
# two steps (ST_RO_CHALT=1, lib_chalt) vs every step (lib_cur: the same
# refactored source, lib_head: the committed one) -- rollout parity + A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05x2
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_chalt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py -m gpu -x -q -k "rollout or soak or long or generation or rewind or twist" --timeout 300 --timeout-method thread > gpurun_out/r05x2/pytest_chalt.log 2>&1 || exit 1
ST_LIB=$B/lib_chalt.so timeout -k 10 150 python tools/ro_stamps.py > gpurun_out/r05x2/ro_stamps_chalt.txt 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_head.so $B/lib_cur.so $B/lib_chalt.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05x2/ab.txt || exit 1
  done
done
