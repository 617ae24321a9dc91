#!/bin/bash
# Round 5: st_step with its first-load operands as preloaded kernel
# arguments (ST_KPRELOAD=1, -amdgpu-kernarg-preload-count=6) -- parity,
# graph-replayed stamps, A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05s
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_kpre.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py tests/test_gpu_vec_env.py tests/test_gpu_wire.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05s/pytest_kpre.log 2>&1 || exit 1
ST_LIB=$B/lib_cur.so timeout -k 10 150 python tools/stamps.py --graph > gpurun_out/r05s/stamps_cur.txt 2>&1 || exit 1
ST_LIB=$B/lib_kpre.so timeout -k 10 150 python tools/stamps.py --graph > gpurun_out/r05s/stamps_kpre.txt 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_cur.so $B/lib_kpre.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05s/ab_kpre.txt || exit 1
  done
done
