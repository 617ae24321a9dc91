# rollout issue-priority variants of the tree's kernel + SQ counters of the tree's kernel
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
B=gym-simpletetris_amd/csrc/build; N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
TAG=${TAG:-ro9}
for n in 65536 32768; do
  for i in 1 2; do
    for lib in $B/lib_base.so $N $B/lib_l2d3.so $B/lib_l3d3.so $B/lib_l0d3.so; do
      AB_N=$n ST_LIB=$lib AB_LABEL="$(basename $lib) n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 || exit 1
    done
  done
done | tee gpurun_out/ab_$TAG.txt
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/sq_$TAG" -o sq -- python3 "$R/tools/ab_rollout.py" 100 5 > /dev/null 2> "$R/gpurun_out/sq_$TAG.err" && python3 "$R/tools/sq_summary.py" "$R/gpurun_out/sq_$TAG/sq_counter_collection.csv" | tee -a "$R/gpurun_out/ab_$TAG.txt"
