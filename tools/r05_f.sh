#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05f
B=gym-simpletetris_amd/csrc/build
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05f/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python tools/ro_stamps.py > gpurun_out/r05f/ro_stamps_base.txt 2>&1 || exit 1
ST_LIB=$R/$B/lib_ldswin.so timeout -k 10 120 python tools/ro_stamps.py > gpurun_out/r05f/ro_stamps_ldswin.txt 2>&1 || exit 1
