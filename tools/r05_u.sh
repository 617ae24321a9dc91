#!/bin/bash
# Round 5: the logic wave's output-pointer kernarg loads hoisted to the
# kernel entry (ST_KA_HOIST=1) + piece word via the stats pointer (lib_kah)
# against the committed preload build (lib_head).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05u
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_kah.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05u/pytest_kah.log 2>&1 || exit 1
for i in 1 2 3 4; do
  for lib in $B/lib_head.so $B/lib_kah.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05u/ab.txt || exit 1
  done
done
