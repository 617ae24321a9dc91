#!/bin/bash
# st_step time vs boards per GPU (C3, packed, eager launches, headline only):
# one JSON line per size -> gpurun_out/nsweep_$TAG.jsonl
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-ns}
for n in ${SIZES:-4096 16384 65536 262144 524288 1048576}; do
  timeout -k 10 180 python bench.py --n-envs $n --steps ${STEPS:-1000} --warmup 50 --no-extras --no-cpu-baseline ${EXTRA} \
    | python -c "
import json, sys
d = json.load(sys.stdin)
r = d['roofline']
print(json.dumps({'n': $n, 'us_per_step': d['ms_per_step'] * 1e3, 'event_us_per_launch': r['event_us_per_launch'],
                  'steady_us': r['steady']['event_us_per_launch'], 'value': d['value'], 'frac': r['frac'],
                  'frac_steady': r['steady']['frac'], 'p_lock': d['p_lock'], 'kernel_source_sha': r['kernel_source_sha']}))" \
    || exit 1
done | tee gpurun_out/nsweep_$TAG.jsonl
