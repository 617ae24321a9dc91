#!/bin/bash
# st_step / st_rollout throughput vs boards per GPU (C3 rewards), bench.py --no-extras
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for n in 4096 16384 65536 262144 524288 1048576 4194304; do
  timeout -k 10 200 python bench.py --n-envs $n --steps 400 --warmup 50 --no-extras 2>/dev/null \
   | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print(json.dumps({'n': $n, 'us_per_step': d['ms_per_step']*1e3, 'kernel_us': r['kernel_us'], 'value': d['value'], 'frac_s8d': r['frac'], 'frac_layout': r['frac_layout'], 'p_lock': d['p_lock']}))" || exit 1
done
