#!/bin/bash
# Round 6: rocprofv3 --kernel-trace --stats of the headline alone launched
# as a hipGraph of K steps (back to back on the GPU) and eagerly (the
# default; host-bound under the tracer), to separate the tracer's
# per-dispatch cost from the kernel.  Output: gpurun_out/r06n/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/r06n"; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o graph -- python3 $R/bench.py --no-extras --no-cpu-baseline --launch graph > "$O/bench_graph.json" 2> "$O/graph.err" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o eager -- python3 $R/bench.py --no-extras --no-cpu-baseline > "$O/bench_eager.json" 2>> "$O/graph.err" \
 && (cd "$R" && python3 tools/trace_summary.py "$O/prof/graph_kernel_trace.csv" > "$O/trace_summary_graph.txt" && python3 tools/trace_summary.py "$O/prof/eager_kernel_trace.csv" > "$O/trace_summary_eager.txt") \
 && find "$O/prof" -name "*kernel_trace.csv" -delete && echo ok
