set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
A=$R/gym-simpletetris_amd/csrc/build/lib_ablation.so
for ab in 0 1 2 3 8 10 0; do
  ST_LIB=$A ST_ABLATE=$ab timeout -k 10 120 python tools/ab_rollout.py 100 20 || exit 1
done | tee gpurun_out/ro_ablate_r03.txt
timeout -k 10 120 python tools/ab_rollout.py 100 20 f32 | tee -a gpurun_out/ro_ablate_r03.txt
