#!/bin/bash
# Round 5 final sources: the driver's command first, its repeats, K = 4,000
# (tools/fresh_lease.sh), then the boards-per-GPU sweep.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
bash tools/fresh_lease.sh r05_final2 || exit 1
TAG=r05_final timeout -k 10 900 bash tools/nsweep.sh > /dev/null || exit 1
