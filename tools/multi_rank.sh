#!/bin/bash
# N>1 bench logic on a one-GPU box: 2 ranks sharing cuda:0 over gloo.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
ST_BENCH_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 200 --warmup 20 \
  --backend gloo --gather --n-envs 16384
