set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for n in 16384 32768 65536 131072 262144 524288; do
  AB_N=$n AB_LABEL="new n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 || exit 1
  AB_N=$n ST_LIB=gym-simpletetris_amd/csrc/build/lib_base.so AB_LABEL="base n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 || exit 1
done | tee gpurun_out/ro_nsweep.txt
