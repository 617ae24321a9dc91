#!/bin/bash
# The driver's bench shape (--steps 20 --warmup 5) repeated on one box, to
# show its run-to-run spread; headline only (--no-extras --no-cpu-baseline).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>/dev/null \
   | python -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'run': $i, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'event_us_per_launch': d['roofline']['event_us_per_launch'], 'steady_us': d['roofline']['steady']['event_us_per_launch']}))" || exit 1
done
