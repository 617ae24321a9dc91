set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
B=gym-simpletetris_amd/csrc/build; N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "rollout or soak or interop or async" > gpurun_out/pytest_ro7.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ro7.log; grep -m3 "^E " gpurun_out/pytest_ro7.log; [ $rc -eq 0 ] || exit $rc
for n in 65536 131072; do
  for i in 1 2; do
    for lib in $B/lib_base.so $N; do
      AB_N=$n ST_LIB=$lib AB_LABEL="$(basename $lib) n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 f32 || exit 1
    done
  done
done | tee gpurun_out/ab_ro7.txt
