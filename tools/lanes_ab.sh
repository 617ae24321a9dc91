#!/bin/bash
# tools/lanes_proto (layout A/B: one env per lane vs 16 lanes per env) at a
# few env counts; each run checks the two layouts against each other first.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for n in 16384 65536 262144; do
  timeout -k 10 120 ./tools/lanes_proto $n 100 20 || exit 1
done | tee gpurun_out/lanes_proto.jsonl
