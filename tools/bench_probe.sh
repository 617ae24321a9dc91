set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
echo "host $(nproc) $(python -c 'import os;print(len(os.sched_getaffinity(0)))')"
for L in graph eager; do for a in "20 5" "20 5" "200 20"; do set -- $a
timeout -k 10 120 python bench.py --gpus 1 --steps $1 --warmup $2 --launch $L --no-extras | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$L', d['steps'], d['warmup'], 'wall %.2f ev %.2f plock %.3f frac %.3f' % (d['ms_per_step']*1e3, d['event_ms_per_step']*1e3, d['p_lock'], r['frac']))" || exit 1
done; done
timeout -k 10 300 python bench.py > gpurun_out/bench_def.json 2> gpurun_out/bench_def.err || exit 1
ST_BENCH_SHARED_GPU=1 timeout -k 10 200 python bench.py --gpus 2 --backend gloo --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || exit 1
echo all ok
