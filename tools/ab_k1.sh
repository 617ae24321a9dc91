set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
B=gym-simpletetris_amd/csrc/build; N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_k1.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_k1.log; grep -m3 -E "^E |FAILED" gpurun_out/pytest_k1.log; [ $rc -eq 0 ] || exit $rc
TAG=k1 bash tools/ab_step_libs.sh 2 $B/lib_base.so $B/lib_none.so $B/lib_nob0.so $B/lib_ovp.so $N
