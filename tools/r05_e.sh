#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05e
B=gym-simpletetris_amd/csrc/build
PRELUDES=1 timeout -k 10 120 python tools/region_probe.py > gpurun_out/r05e/region_preludes.jsonl || exit 1
TAG=r05e_ab_rows8 timeout -k 10 600 bash tools/ab.sh step 3 $B/lib_base.so gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e/pytest_gpu.log 2>&1 || exit 1
