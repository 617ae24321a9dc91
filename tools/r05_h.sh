#!/bin/bash
# Round 5: phase stamps of the hot-row + cold-record layout (compare with
# profiles/r04/stamps_final.txt, the SoA layout) and of the rollout.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05h
timeout -k 10 150 python tools/stamps.py > gpurun_out/r05h/stamps_new.txt 2>&1 || exit 1
timeout -k 10 150 python tools/stamps.py --graph > gpurun_out/r05h/stamps_new_graph.txt 2>&1 || exit 1
timeout -k 10 150 python tools/ro_stamps.py > gpurun_out/r05h/ro_stamps_new.txt 2>&1 || exit 1
