#!/bin/bash
# st_step time vs envs per GPU (waves per SIMD: 32768 = 0.5, 65536 = 1, 131072 = 2, 262144 = 4).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-ns}
for n in 16384 32768 65536 131072 262144; do
  timeout -k 10 120 python bench.py --n-envs $n --steps 1000 --warmup 50 --no-extras --no-cpu-baseline ${EXTRA} \
    | python -c "import json,sys; d=json.load(sys.stdin); print('n=$n', 'us/step=%.3f' % (d['ms_per_step']*1e3), 'kernel_us=%.3f' % d['roofline']['kernel_us'], 'env-steps/s=%.3e' % d['value'])" \
    || exit 1
done | tee gpurun_out/nsweep_$TAG.txt
