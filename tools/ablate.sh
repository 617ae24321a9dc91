#!/bin/bash
# Timing-only ablations of the step kernel (results are NOT valid games).
# AB_BITS="0 1024 0 1024" picks the ST_ABLATE values (st_internal.h, KParams::ablate).
# Needs the ablation build (the product kernels compile the ablations out):
#   make -C gym-simpletetris_amd/csrc variant V=ablation DEFS=-DST_ABLATION=1
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
export ST_LIB="${ST_LIB:-$R/gym-simpletetris_amd/csrc/build/lib_ablation.so}"
TAG=${TAG:-abl}
for ab in ${AB_BITS:-0 1 2 4 8 3 0}; do
  ST_ABLATE=$ab timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline ${EXTRA:---steps 500 --warmup 50} \
    | python -c "import json,sys; d=json.load(sys.stdin); print('ablate=$ab', 'us/step=%.3f' % (d['ms_per_step']*1e3), 'event_us=%.3f steady_us=%.3f' % (d['roofline']['event_us_per_launch'], d['roofline']['steady']['event_us_per_launch']))" \
    || exit 1
done | tee gpurun_out/ablate_$TAG.txt
