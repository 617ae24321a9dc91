#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05h
B=$R/gym-simpletetris_amd/csrc/build
NEW=$R/gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
ST_LIB=$B/lib_base.so timeout -k 10 150 python tools/stamps.py > gpurun_out/r05h/stamps_base.txt 2>&1 || exit 1
ST_LIB=$NEW timeout -k 10 150 python tools/stamps.py > gpurun_out/r05h/stamps_new.txt 2>&1 || exit 1
