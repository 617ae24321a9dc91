# rollout A/B: previous commit's kernels (lib_base) vs the tree's library,
# after the rollout parity tests; then the tree's rollout stamps
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
B=gym-simpletetris_amd/csrc/build; N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
TAG=${TAG:-ro8}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "rollout or soak" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_$TAG.log; grep -m3 "^E " gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for n in 65536 32768; do
  for i in 1 2; do
    for lib in $B/lib_base.so $N; do
      AB_N=$n ST_LIB=$lib AB_LABEL="$(basename $lib) n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 f32 || exit 1
    done
  done
done | tee gpurun_out/ab_$TAG.txt
timeout -k 10 120 python tools/ro_stamps.py 100 6 > gpurun_out/ro_stamps_$TAG.txt 2>&1
