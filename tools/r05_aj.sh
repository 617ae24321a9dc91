#!/bin/bash
# Round 5: the rollout draw wave publishing its queue counter without the
# release fence's lgkmcnt(0) wait (ST_FD_NOFENCE=1, lib_nof) vs with it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05aj
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_nof.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py -m gpu -x -q -k "rollout or soak or long or generation or rewind or twist" --timeout 300 --timeout-method thread > gpurun_out/r05aj/pytest_nof.log 2>&1 || exit 1
ST_LIB=$B/lib_nof.so timeout -k 10 150 python tools/ro_stamps.py > gpurun_out/r05aj/ro_stamps_nof.txt 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_nof.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 1000)" >> gpurun_out/r05aj/ab.txt || exit 1
  done
done
