#!/bin/bash
# Round 5: reward / done stores non-temporal (ST_RD_CPOL=2) in st_step and
# the rollout output wave, against the committed build (lib_head).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05v
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_rdnt.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "rollout or oracle or wire or vec" -x -q --timeout 300 --timeout-method thread > gpurun_out/r05v/pytest_rdnt.log 2>&1 || exit 1
for i in 1 2 3 4; do
  for lib in $B/lib_head.so $B/lib_rdnt.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05v/ab.txt || exit 1
  done
done
