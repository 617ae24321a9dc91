#!/bin/bash
# GPU parity tests + a short bench (all variants) + SQ instruction counters.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-q}
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_$TAG.log; grep -m3 "^E " gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 500 --warmup 50 --no-cpu-baseline \
 | python -c "import json,sys; d=json.load(sys.stdin); v=d['variants']; print('step=%.3f step_f32=%.3f rollout_packed=%.3f rollout_f32=%.3f us/step; frac step %.3f f32 %.3f ro %.3f rof32 %.3f' % (d['ms_per_step']*1e3, v['step_f32']['ms_per_step']*1e3, v['rollout_packed']['ms_per_step']*1e3, v['rollout_f32']['ms_per_step']*1e3, d['roofline']['frac'], v['step_f32']['roofline']['frac'], v['rollout_packed']['roofline']['frac'], v['rollout_f32']['roofline']['frac']))" || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_sq_$TAG" -o sq -- python3 "$R/bench.py" --steps 100 --warmup 10 --no-graph --no-cpu-baseline --rollout-chunk 50 > /dev/null 2> "$R/gpurun_out/pmc_sq_$TAG.err" || exit 1
cd "$R" && python3 tools/sq_summary.py "gpurun_out/pmc_sq_$TAG/sq_counter_collection.csv"
