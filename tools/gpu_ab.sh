#!/bin/bash
# One GPU call: the -m gpu suite on the in-tree library, the parity files on a
# candidate build (CAND=lib.so: tests/test_gpu_parity.py, long horizon,
# vec env, wire), then tools/ab.sh step / rollout over the libraries named on
# the command line (the in-tree one first).  Test failures (pytest rc 1) do
# not stop the A/B; a crash, abort, fault or time limit ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
mkdir -p gpurun_out; TAG=${TAG:-r04}; ROUNDS=${ROUNDS:-3}
N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
rc=0
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -m5 -E "^(E |FAILED)" gpurun_out/pytest_gpu_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "$CAND" ]; then
  ST_LIB="$CAND" timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_long_horizon.py tests/test_gpu_vec_env.py tests/test_gpu_wire.py \
    > gpurun_out/pytest_cand_$TAG.log 2>&1; rc2=$?
  echo "candidate parity:"; tail -2 gpurun_out/pytest_cand_$TAG.log; grep -m5 -E "^(E |FAILED)" gpurun_out/pytest_cand_$TAG.log
  [ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
fi
# STEP_LIBS / RO_LIBS (space-separated) override the command-line list per mode
TAG=ab_step_$TAG bash tools/ab.sh step "$ROUNDS" "$N" ${STEP_LIBS:-"$@"} || exit $?
TAG=ab_ro_$TAG bash tools/ab.sh rollout "$ROUNDS" "$N" ${RO_LIBS:-"$@"} || exit $?
exit $rc
