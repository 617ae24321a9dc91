#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd /tmp; export TMPDIR=/tmp
O="$R/gpurun_out"; mkdir -p "$O"; TAG=${TAG:-d1}
B="python3 $R/bench.py --no-cpu-baseline --no-extras"
for n in 65536 131072 262144 524288; do
  timeout -k 10 120 $B --steps 300 --warmup 30 --n-envs $n | python3 -c "import json,sys; d=json.load(sys.stdin); print('n=$n us/step=%.3f Gsteps/s=%.2f' % (d['ms_per_step']*1e3, d['value']/1e9))" || exit 1
done | tee "$O/occupancy_$TAG.txt"
timeout -k 10 60 rocprofv3 -L > "$O/counters_$TAG.txt" 2>&1 || true
grep -o "SQ_[A-Z_]*" "$O/counters_$TAG.txt" | sort -u | tr '\n' ' ' | head -c 3000; echo
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$O/pmc_sq_$TAG" -o sq -- $B --steps 100 --warmup 10 --no-graph > /dev/null 2> "$O/pmc_sq_$TAG.err" && echo "sq ok"
