#!/bin/bash
# A second rocprofv3 --kernel-trace --stats pass of the headline alone on
# another box (TAG=r05b): the traced duration's box-to-box spread
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-r05b}
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o head -- python3 "$R/bench.py" --no-extras > "$O/prof_head_$TAG.json" 2> "$O/prof_$TAG.err" \
 && (cd "$R" && python3 tools/trace_summary.py "$O/prof_$TAG/head_kernel_trace.csv" > "$O/trace_summary_head_$TAG.txt") \
 && find "$O/prof_$TAG" -name "*.csv" ! -name "*_stats.csv" -delete \
 && echo "trace ok" && head -12 "$O/trace_summary_head_$TAG.txt"
