#!/bin/bash
# Round 5: tools/ro_gap.py -- rollout timing on engines built / aged as the
# bench and as the A/B harness build them.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05al
timeout -k 10 300 python tools/ro_gap.py > gpurun_out/r05al/ro_gap.txt 2>&1 || exit 1
KINDS="plain sharded" timeout -k 10 300 python tools/ro_gap.py >> gpurun_out/r05al/ro_gap.txt 2>&1 || exit 1
