#!/bin/bash
# Round 5: kernarg-preload follow-ups -- the logic wave's piece word from the
# preloaded stats pointer (lib_kpw), plus the post-B0 kernel arguments forced
# into SGPRs early (lib_kasm), against the committed preload build (lib_head).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05t
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_kpw.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05t/pytest_kpw.log 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_head.so $B/lib_kpw.so $B/lib_kasm.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05t/ab.txt || exit 1
  done
done
