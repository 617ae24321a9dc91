#!/bin/bash
# Round 5: the bench's rollout vs the harness's -- HIP_FORCE_DEV_KERNARG
# (bench.py sets 1, the harness leaves HIP's default) on both.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05ab
O=gpurun_out/r05ab
for kv in 0 1; do
  echo "harness kernarg=$kv $(HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 120 python tools/ab_step.py 1000)" >> $O/ro.txt || exit 1
  echo "bench kernarg=$kv $(HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 python bench.py --no-cpu-baseline --no-surfaces --steps 1000 --warmup 100 | python -c "import json,sys; d=json.load(sys.stdin); r=d['variants']['rollout_packed']; print(r['ms_per_step']*1e3, r['roofline']['event_us_per_launch'], d['ms_per_step']*1e3)")" >> $O/ro.txt || exit 1
done
