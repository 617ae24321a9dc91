#!/bin/bash
# Round 5: graph-replayed phase stamps, round-5 start layout (ab/base: that
# commit's package + lib_base.so) vs the current tree.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05k
for i in 1 2; do
  timeout -k 10 150 python ab/base/tools/stamps.py --graph > gpurun_out/r05k/stamps_graph_base_$i.txt 2>&1 || exit 1
  timeout -k 10 150 python tools/stamps.py --graph > gpurun_out/r05k/stamps_graph_new_$i.txt 2>&1 || exit 1
done
