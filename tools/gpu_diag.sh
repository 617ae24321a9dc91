#!/bin/bash
# Diagnostics of the in-tree kernels in one GPU call (TAG=r04 bash tools/gpu_diag.sh):
# st_step and st_rollout phase stamps (ST_STAMPS builds of the same sources)
# and SQ instruction / wait counters (one rocprofv3 --pmc pass each).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; TAG=${TAG:-r04}
timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ro_stamps.py > gpurun_out/ro_stamps_$TAG.txt 2>&1 || exit $?
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv \
   -d "$R/gpurun_out/sq_step_$TAG" -o sq -- python3 "$R/bench.py" --no-extras --no-cpu-baseline --steps 200 --warmup 20 \
   > /dev/null 2> "$R/gpurun_out/sq_step_$TAG.err") || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv \
   -d "$R/gpurun_out/sq_ro_$TAG" -o sq -- python3 "$R/tools/ab_rollout.py" 100 5 \
   > /dev/null 2> "$R/gpurun_out/sq_ro_$TAG.err") || exit $?
python3 tools/sq_summary.py gpurun_out/sq_step_$TAG/sq_counter_collection.csv > gpurun_out/sq_summary_$TAG.txt
python3 tools/sq_summary.py gpurun_out/sq_ro_$TAG/sq_counter_collection.csv >> gpurun_out/sq_summary_$TAG.txt
find gpurun_out/sq_step_$TAG gpurun_out/sq_ro_$TAG -name "*.csv" -delete
cat gpurun_out/stamps_$TAG.txt gpurun_out/ro_stamps_$TAG.txt gpurun_out/sq_summary_$TAG.txt
