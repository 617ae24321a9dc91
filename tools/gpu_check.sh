#!/bin/bash
# One gpurun call: GPU parity tests, smoke, the default bench.  Every GPU step
# has its own time limit; steps are chained with && so a failure (fault,
# abort, timeout) ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
echo "== host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" | tee gpurun_out/host_$TAG.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
 && echo "bench ok" \
 && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20_$TAG.json 2>> gpurun_out/bench_$TAG.err \
 && echo "bench k20 ok"
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
exit $rc
