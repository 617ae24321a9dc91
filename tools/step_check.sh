#!/bin/bash
# Full GPU suite, then the st_step A/B against build/lib_base.so (the
# round-start library): bench.py --no-extras at K = 2000 and K = 20, 3
# alternating rounds (tools/ab_step_libs.sh).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-stepc}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_$TAG.log; grep -m5 "^E " gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
TAG=$TAG bash tools/ab_step_libs.sh 3 gym-simpletetris_amd/csrc/build/lib_base.so gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
