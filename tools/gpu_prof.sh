#!/bin/bash
# Profiling pass for one round's numbers (TAG=r04 bash tools/gpu_prof.sh):
#  1. rocprofv3 --kernel-trace --stats of the default bench command (all
#     variants) and of the headline alone (--no-extras: clean per-kernel stats),
#     plus tools/trace_summary.py per-run splits of both traces and their
#     per-kernel@grid@k JSON (with each key's p_lock from the traced run's
#     own bench line) -> profiles/${TAG}_trace.json on the box (so a bench
#     run after it in the same call reports roofline.rocprof) and gpurun_out/
#  2. PMC: FETCH_SIZE and WRITE_SIZE in SEPARATE passes (TCC slot limits) over
#     eager launches of every kernel variant (not the Python-surface timings,
#     whose launches of the same kernels would mix into the averages), plus
#     the same two passes over
#     tools/pmc_calib (known byte counts) -> tools/pmc_summary.py ->
#     gpurun_out/${TAG}_pmc.json (copy to profiles/)
# Every GPU step has its own time limit; steps are chained with &&.  The raw
# trace / counter CSVs are deleted once summarised (gpurun copies back at most
# 64 MiB of gpurun_out/).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-r04}
O="$R/gpurun_out"
mkdir -p "$O"
B="$R/bench.py"
run() { echo "== $*"; timeout -k 10 400 "$@"; }
run rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o full -- python3 $B --no-cpu-baseline > "$O/prof_bench_$TAG.json" 2> "$O/prof_$TAG.err" \
 && run rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o head -- python3 $B --no-extras > "$O/prof_head_$TAG.json" 2>> "$O/prof_$TAG.err" \
 && run rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/pmc_fetch_$TAG" -o packed -- python3 $B --no-cpu-baseline --no-surfaces --steps 600 --warmup 100 --launch eager > "$O/pmc_fetch_bench_$TAG.json" 2>> "$O/prof_$TAG.err" \
 && run rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/pmc_write_$TAG" -o packed -- python3 $B --no-cpu-baseline --no-surfaces --steps 600 --warmup 100 --launch eager > "$O/pmc_write_bench_$TAG.json" 2>> "$O/prof_$TAG.err" \
 && run rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/pmc_cal_fetch_$TAG" -o cal -- "$R/tools/pmc_calib" >> "$O/prof_$TAG.err" 2>&1 \
 && run rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/pmc_cal_write_$TAG" -o cal -- "$R/tools/pmc_calib" >> "$O/prof_$TAG.err" 2>&1 \
 && (cd "$R" && python3 tools/pmc_summary.py "$TAG" "$O/pmc_fetch_$TAG" "$O/pmc_write_$TAG" "$O/pmc_cal_fetch_$TAG" "$O/pmc_cal_write_$TAG" --rollout-k 100 --bench-json "$O/pmc_fetch_bench_$TAG.json" > "$O/pmc_summary_$TAG.json" && cp "profiles/${TAG}_pmc.json" "$O/") \
 && (cd "$R" && python3 tools/trace_summary.py "$O/prof_$TAG/full_kernel_trace.csv" > "$O/trace_summary_$TAG.txt" \
     && python3 tools/trace_summary.py "$O/prof_$TAG/head_kernel_trace.csv" > "$O/trace_summary_head_$TAG.txt" \
     && python3 tools/trace_summary.py --json "$TAG" --rollout-k 100 "$O/prof_$TAG/head_kernel_trace.csv:$O/prof_head_$TAG.json" "$O/prof_$TAG/full_kernel_trace.csv:$O/prof_bench_$TAG.json" > "profiles/${TAG}_trace.json" \
     && cp "profiles/${TAG}_trace.json" "$O/") \
 && find "$O/prof_$TAG" "$O/pmc_fetch_$TAG" "$O/pmc_write_$TAG" "$O/pmc_cal_fetch_$TAG" "$O/pmc_cal_write_$TAG" \
      -name "*.csv" ! -name "*_stats.csv" -delete \
 && echo "prof ok"
