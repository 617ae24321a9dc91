#!/bin/bash
# One GPU call of a round's check + A/B (TAG=r04b bash tools/gpu_round.sh lib...):
#  1. the -m gpu suite on the in-tree library, then smoke;
#  2. tools/ab.sh step over the libraries named on the command line and the
#     in-tree one (ROUNDS alternating rounds, K = 2000 and the driver's 20);
#  3. the default bench line and the driver's shape.
# Test FAILURES (pytest rc 1) do not stop the A/B (its numbers stay useful);
# a crash, abort, fault or time limit (any other non-zero rc) ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
mkdir -p gpurun_out; TAG=${TAG:-r04}; ROUNDS=${ROUNDS:-2}
N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
echo "== host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" > gpurun_out/host_$TAG.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log; grep -m5 -E "^(E |FAILED)" gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
echo "smoke ok"
if [ $# -gt 0 ]; then
  TAG=ab_$TAG bash tools/ab.sh step "$ROUNDS" "$@" "$N" || exit $?
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
echo "bench ok"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20_$TAG.json \
  2>> gpurun_out/bench_$TAG.err || exit $?
echo "bench k20 ok"
exit $rc
