#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for lib in "" "$R/gym-simpletetris_amd/csrc/build/libsimpletetris_noring.so" "" "$R/gym-simpletetris_amd/csrc/build/libsimpletetris_noring.so"; do
  ST_LIB="$lib" timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-cpu-baseline \
   | python -c "import json,sys; d=json.load(sys.stdin); v=d['variants']; print('lib=%s step=%.3f rollout_packed=%.3f rollout_f32=%.3f us/step' % ('${lib##*/}' or 'ring', d['ms_per_step']*1e3, v['rollout_packed']['ms_per_step']*1e3, v['rollout_f32']['ms_per_step']*1e3))" || exit 1
done
