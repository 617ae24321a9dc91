#!/bin/bash
# Timing-only ablations of the queued-draw st_rollout (results are NOT valid
# games), 65,536 envs, 100-step launches: 0 = none, 1 = no lock path, 2 = no
# draws, 8 = no obs output, 16 = no next-generation chunk, 32 = the logic
# wave never waits for the draw / output waves, 64 = no reward / done / episode-counter stores in the logic wave, 128 = the logic wave never waits for the draw wave (fd), 256 = never for the output wave (fq).
# Needs: make -C gym-simpletetris_amd/csrc variant V=ablation DEFS=-DST_ABLATION=1
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
A=$R/gym-simpletetris_amd/csrc/build/lib_ablation.so
TAG=${TAG:-roq}
for ab in 0 32 64 128 256 0; do
  AB_LABEL="ablate=$ab" ST_LIB=$A ST_ABLATE=$ab timeout -k 10 120 python tools/ab_rollout.py 100 10 || exit 1
done | tee gpurun_out/roq_ablate_$TAG.txt
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for lib in "$R/gym-simpletetris_amd/csrc/build/lib_base.so" "$R/gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so"; do
  b=$(basename $lib .so)
  ST_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/sq_${TAG}_$b" -o sq -- python3 "$R/tools/ab_rollout.py" 100 5 > /dev/null 2> "$R/gpurun_out/sq_${TAG}_$b.err" || exit 1
  echo "$b:" | tee -a "$R/gpurun_out/roq_ablate_$TAG.txt"
  python3 "$R/tools/sq_summary.py" "$R/gpurun_out/sq_${TAG}_$b/sq_counter_collection.csv" | tee -a "$R/gpurun_out/roq_ablate_$TAG.txt"
done
