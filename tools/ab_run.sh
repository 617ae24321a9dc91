#!/bin/bash
# usage: tools/ab_run.sh lib1.so lib2.so ... (3 alternating rounds of tools/ab_step.py)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for round in 1 2 3; do
  for lib in "$@"; do
    ST_LIB="$lib" timeout -k 10 120 python tools/ab_step.py ${K:-2000} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
