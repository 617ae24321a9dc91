#!/bin/bash
# A/B under the tracer: st_step's reward/done (kRD) and state (kST) store
# policy, nt (head) vs write-back, rocprofv3 --kernel-trace of the headline
# alone plus an untraced headline line, alternating on one box
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/tpa"; mkdir -p "$O"
P="$R/gym-simpletetris_amd/gym_simpletetris_amd"
for rep in 1 2; do
  for v in head rdwb allwb; do
    if [ $v = head ]; then L="$P/libsimpletetris.so"; else L="$P/lib_$v.so"; fi
    ST_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/p_${v}_$rep" -o head -- python3 "$R/bench.py" --no-extras > "$O/t_${v}_$rep.json" 2> "$O/t_${v}_$rep.err" || exit $?
    (cd "$R" && python3 tools/trace_summary.py "$O/p_${v}_$rep/head_kernel_trace.csv" > "$O/s_${v}_$rep.txt") || exit $?
    find "$O/p_${v}_$rep" -name "*.csv" -delete
    ST_LIB=$L timeout -k 10 120 python3 "$R/bench.py" --no-extras > "$O/u_${v}_$rep.json" 2> "$O/u_${v}_$rep.err" || exit $?
    python3 - "$v" "$O/s_${v}_$rep.txt" "$O/u_${v}_$rep.json" <<'PY'
import json, sys
tr = [l for l in open(sys.argv[2]) if "k_step" in l and " 4000 " in l]
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print("%-6s traced(4000): %s | untraced %.3f us steady %.3f" % (sys.argv[1], " ".join(tr[0].split()[-5:-3]) if tr else "?",
      d["ms_per_step"] * 1e3, d["roofline"]["steady"]["event_us_per_launch"]), flush=True)
PY
  done
done
