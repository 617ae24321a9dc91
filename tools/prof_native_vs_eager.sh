#!/bin/bash
# Round 6: the headline traced (rocprofv3 --kernel-trace --stats) under the
# native launch loop (st_step_n) and eager ctypes launches, one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/r06z"; mkdir -p "$O"
for m in native eager; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o $m -- python3 $R/bench.py --no-extras --no-cpu-baseline --launch $m > "$O/bench_$m.json" 2>> "$O/err.txt" || exit 1
(cd "$R" && python3 tools/trace_summary.py "$O/prof/${m}_kernel_trace.csv" > "$O/trace_summary_$m.txt") || exit 1
done
find "$O/prof" -name "*kernel_trace.csv" -delete; echo ok
