#!/bin/bash
# One parameterised A/B driver over library builds (replaces round 3's
# one-off ab_ro*.sh / roq_*.sh / ab_*_libs.sh scripts).  Libraries alternate
# within each round, so box drift hits every build alike.
#
# usage: tools/ab.sh MODE ROUNDS lib.so [lib.so ...]
#   MODE step     bench.py --no-extras (eager st_step, 65,536 envs, C3) at
#                 K = 2000 and at the driver's K = 20
#   MODE rollout  tools/ab_rollout.py (st_rollout, CH-step launches)
#   MODE bench    bench.py with all variants (step, f32, rollouts)
#   MODE stamps   tools/stamps.py phase split (stamp builds: ST_STAMPS=1)
# env: TAG (output name), AB_N (envs, rollout), AB_F32=1 (rollout f32 too),
#      CH / L (rollout steps per launch / launches), STEPS / WARMUP (bench),
#      SQ=1 (rollout/step: SQ instruction counters of the FIRST library after
#      the rounds, one rocprofv3 --pmc pass of its own)
# Variant builds: make -C gym-simpletetris_amd/csrc variant V=name DEFS="-D..."
#   -> gym-simpletetris_amd/csrc/build/lib_name.so
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
MODE=$1; ROUNDS=$2; shift 2
TAG=${TAG:-ab_$MODE}
OUT="gpurun_out/$TAG.txt"
: > "$OUT"
one() {  # one timing of library $1
  local lib=$1 name; name=$(basename "$lib")
  case "$MODE" in
  step)
    for K in 2000 20; do
      W=100; [ $K -eq 20 ] && W=5
      ST_LIB="$lib" timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --steps $K --warmup $W \
        | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('%-20s K=%-5d us_per_step=%.3f event_us=%.3f steady_us=%.3f value=%.4g' % ('$name', $K, d['ms_per_step']*1e3, r['event_us_per_launch'], r['steady']['event_us_per_launch'], d['value']))" || return 1
    done ;;
  rollout)
    AB_N=${AB_N:-65536} ST_LIB="$lib" AB_LABEL="$name n=${AB_N:-65536}" \
      timeout -k 10 120 python tools/ab_rollout.py ${CH:-100} ${L:-10} ${AB_F32:+f32} || return 1 ;;
  bench)
    ST_LIB="$lib" timeout -k 10 200 python bench.py --steps ${STEPS:-500} --warmup ${WARMUP:-50} --no-cpu-baseline \
      | python -c "import json,sys; d=json.load(sys.stdin); v=d['variants']; print('%-20s step=%.3f step_f32=%.3f rollout_packed=%.3f rollout_f32=%.3f us/step' % ('$name', d['ms_per_step']*1e3, v['step_f32']['ms_per_step']*1e3, v['rollout_packed']['ms_per_step']*1e3, v['rollout_f32']['ms_per_step']*1e3))" || return 1 ;;
  stamps)
    echo "== $name"; ST_LIB="$lib" timeout -k 10 200 python tools/stamps.py || return 1 ;;
  *) echo "unknown mode $MODE"; return 2 ;;
  esac
}
for i in $(seq "$ROUNDS"); do
  for lib in "$@"; do one "$lib" || exit 1; done
done | tee -a "$OUT" || exit 1
if [ -n "$SQ" ] && [ "$MODE" = rollout -o "$MODE" = step ]; then
  C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  if [ "$MODE" = rollout ]; then P=("$R/tools/ab_rollout.py" 100 5); else P=("$R/bench.py" --no-extras --no-cpu-baseline --steps 200 --warmup 20); fi
  (cd /tmp && export TMPDIR=/tmp && ST_LIB="$1" timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv \
     -d "$R/gpurun_out/sq_$TAG" -o sq -- python3 "${P[@]}" > /dev/null 2> "$R/gpurun_out/sq_$TAG.err") \
    && python3 tools/sq_summary.py "gpurun_out/sq_$TAG/sq_counter_collection.csv" | tee -a "$OUT"
fi
