#!/bin/bash
# A/B: the board / counter rows in coarse-grained (default), fine-grained (1)
# or uncached (3) device memory (ST_STATE_MEMFLAGS), headline bench line,
# alternating runs on one box
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/mf
for rep in 1 2; do
  for f in 0 1 3; do
    ST_STATE_MEMFLAGS=$f timeout -k 10 120 python bench.py --no-surfaces --no-clear-heavy > gpurun_out/mf/b_${f}_$rep.json 2> gpurun_out/mf/b_${f}_$rep.err || exit $?
    python - "$f" gpurun_out/mf/b_${f}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print("flags", sys.argv[1], "value %.4g" % d["value"], "us %.3f" % (d["ms_per_step"] * 1e3), "steady %.3f" % r["steady"]["event_us_per_launch"],
      "rollout %.3f" % (d["variants"]["rollout_packed"]["ms_per_step"] * 1e3), "c4 %.3f" % (d["variants"]["c4"]["ms_per_step"] * 1e3), flush=True)
PY
  done
done
