#!/bin/bash
# SQ instruction / cycle counters of st_rollout (packed, 65,536 envs, 100
# steps per launch) for the product build and the ablation build's
# no-lock-path+no-draw (3) and no-draw (2) variants: per-wave instruction
# counts per launch -> tools/sq_summary.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out"; mkdir -p "$O"; TAG=${TAG:-ro}
A=$R/gym-simpletetris_amd/csrc/build/lib_ablation.so
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
run() { v=$1; shift; echo "== $v"; timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/sq_${TAG}_$v" -o sq -- python3 "$R/tools/ab_rollout.py" 100 5 > /dev/null 2> "$O/sq_${TAG}_$v.err" && python3 "$R/tools/sq_summary.py" "$O/sq_${TAG}_$v/sq_counter_collection.csv"; }
run prod && ST_LIB=$A ST_ABLATE=3 run abl3 && ST_LIB=$A ST_ABLATE=2 run abl2 && ST_LIB=$A ST_ABLATE=1 run abl1
