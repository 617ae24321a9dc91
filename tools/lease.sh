#!/bin/bash
# One parameterised GPU lease script (round 6; replaces round 5's single-use
# tools/r05_*.sh wrappers).  Each argument is one step "SECONDS|NAME|COMMAND":
# the steps run in order from the repo root, each under its own time limit
# (timeout -k 10), stdout + stderr to gpurun_out/$TAG/NAME.log; the first
# step that fails, faults or times out ends the call (no retries).
#   gpurun --timeout 900 -- bash tools/lease.sh r06a \
#     "600|pytest|python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread" \
#     "300|bench|python bench.py"
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" || exit 2
export TMPDIR=/tmp
TAG=$1; shift
O="gpurun_out/$TAG"; mkdir -p "$O"
for step in "$@"; do
  secs=${step%%|*}; rest=${step#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc $(( $(date +%s) - start )) s"
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ]; then
    grep -m5 -E "^(E |FAILED)" "$O/$name.log"
    exit $rc
  fi
done
