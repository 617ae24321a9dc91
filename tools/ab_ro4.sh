set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
B=gym-simpletetris_amd/csrc/build
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "rollout or soak or interop" > gpurun_out/pytest_ro4.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ro4.log; grep -m3 "^E " gpurun_out/pytest_ro4.log; [ $rc -eq 0 ] || exit $rc
TAG=ro4 bash tools/ab_libs_ro.sh 3 $B/lib_base.so $B/lib_l3d2.so gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so && \
timeout -k 10 120 python tools/ro_stamps.py 100 6 | tee gpurun_out/ro_stamps_ro4.txt
