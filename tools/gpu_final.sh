#!/bin/bash
# GPU check + bench lines (TAG=r04 bash tools/gpu_final.sh): the -m gpu suite, smoke, the default
# bench (K = 4,000) and the driver's shape (K = 20).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
mkdir -p gpurun_out; TAG=${TAG:-r04}
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
 && echo "bench ok" \
 && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20_$TAG.json 2>> gpurun_out/bench_$TAG.err \
 && echo "bench k20 ok"
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
grep -m5 -E "^(E |FAILED)" gpurun_out/pytest_gpu_$TAG.log
exit $rc
