set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for i in 1 2 3 4; do
  for L in eager graph; do
    ST_BENCH_DEBUG=1 timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 5 --launch $L 2> gpurun_out/k20_dbg_err.txt \
      | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$L K=20 wall_us=%.3f event_us=%.3f steady_us=%.3f value=%.4g' % (d['ms_per_step']*1e3, r['event_us_per_launch'], r['steady']['event_us_per_launch'], d['value']))" || exit 1
    grep timed gpurun_out/k20_dbg_err.txt | head -3
  done
done | tee gpurun_out/k20_dbg.txt
