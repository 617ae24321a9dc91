#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for ab in 0 16 0 16; do
  ST_ABLATE=$ab timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-cpu-baseline --no-extras \
   | python -c "import json,sys; d=json.load(sys.stdin); print('ablate=$ab step=%.3f us' % (d['ms_per_step']*1e3))" || exit 1
done
