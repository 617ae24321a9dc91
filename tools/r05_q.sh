#!/bin/bash
# Round 5: st_step's next-generation chunk stored right after the window
# loads instead of after the draws (ST_CHUNK_EARLY=1); the draw wave's MT
# word / count stored by the logic wave (ST_DSTORE_L=1) -- parity + A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05q
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_both.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05q/pytest_both.log 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_chke.so $B/lib_dsl.so $B/lib_both.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05q/ab_chke.txt || exit 1
  done
done
