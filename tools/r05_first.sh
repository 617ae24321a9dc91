#!/bin/bash
# Round 5's first GPU call: the driver's bench command on the fresh lease
# first (tools/fresh_lease.sh), then the traffic ablations that bound the
# AoS cold-record refactor (timing only, tools/ablate.sh), then the wire tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
bash tools/fresh_lease.sh r05a || exit 1
AB_BITS="0 1024 9216 11264 15360 4096 2048 0" TAG=r05_traffic EXTRA="--steps 2000 --warmup 100" \
  timeout -k 10 400 bash tools/ablate.sh || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wire.py \
  > gpurun_out/r05a/pytest_wire.log 2>&1 || exit 1
