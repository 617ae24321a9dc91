#!/bin/bash
# Round 5: the rollout logic wave publishing its lock mask counter without
# the release fence's lgkmcnt(0) wait (ST_FL_NOFENCE=1, lib_flnf) vs with it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ak
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_flnf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py -m gpu -x -q -k "rollout or soak or long or generation or rewind or twist" --timeout 300 --timeout-method thread > gpurun_out/r05ak/pytest_flnf.log 2>&1 || exit 1
ST_LIB=$B/lib_flnf.so timeout -k 10 150 python tools/ro_stamps.py > gpurun_out/r05ak/ro_stamps_flnf.txt 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_flnf.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05ak/ab.txt || exit 1
  done
done
