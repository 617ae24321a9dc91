#!/bin/bash
# Profiling pass (run after tools/gpu_check.sh in the same gpurun call or alone):
#  - rocprofv3 --kernel-trace --stats of a short bench run (all variants)
#  - PMC: FETCH_SIZE and WRITE_SIZE in SEPARATE passes (TCC slot limits), eager
#    launches, plus the same two passes over tools/pmc_calib (known byte counts)
#  - tools/pmc_summary.py -> profiles/${TAG}_pmc.json
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-r01}
O="$R/gpurun_out"
mkdir -p "$O"
B="python3 $R/bench.py --no-cpu-baseline"
# PMC passes: eager launches, all variants (st_step packed/f32, st_rollout packed/f32)
run() { echo "== $*"; timeout -k 10 300 "$@"; }
run rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o packed -- $B > "$O/prof_bench_$TAG.json" 2> "$O/prof_$TAG.err" \
 && run rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/pmc_fetch_$TAG" -o packed -- $B --steps 600 --warmup 100 --no-graph --rollout-chunk 50 > /dev/null 2>> "$O/prof_$TAG.err" \
 && run rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/pmc_write_$TAG" -o packed -- $B --steps 600 --warmup 100 --no-graph --rollout-chunk 50 > /dev/null 2>> "$O/prof_$TAG.err" \
 && run rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/pmc_cal_fetch_$TAG" -o cal -- "$R/tools/pmc_calib" >> "$O/prof_$TAG.err" 2>&1 \
 && run rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/pmc_cal_write_$TAG" -o cal -- "$R/tools/pmc_calib" >> "$O/prof_$TAG.err" 2>&1 \
 && (cd "$R" && python3 tools/pmc_summary.py "$TAG" "$O/pmc_fetch_$TAG" "$O/pmc_write_$TAG" "$O/pmc_cal_fetch_$TAG" "$O/pmc_cal_write_$TAG" > "$O/pmc_summary_$TAG.json" && cp "profiles/${TAG}_pmc.json" "$O/") \
 && (cd "$R" && python3 tools/trace_summary.py "$O/prof_$TAG/packed_kernel_trace.csv" > "$O/trace_summary_$TAG.txt") \
 && echo "prof ok"
