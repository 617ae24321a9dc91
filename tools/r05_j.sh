#!/bin/bash
# Round 5: cold-record stores merged + atomic count increment (no count reads
# on the common draw path) -- GPU suite, A/B vs the round-5 start layout and
# the first cold-record build, stamps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05j
B=$R/gym-simpletetris_amd/csrc/build
NEW=$R/gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05j/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_base.so $B/lib_aos1.so $NEW; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05j/ab_layout.txt || exit 1
  done
done
timeout -k 10 150 python tools/stamps.py > gpurun_out/r05j/stamps_new.txt 2>&1 || exit 1
