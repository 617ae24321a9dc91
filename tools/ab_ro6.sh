set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
B=gym-simpletetris_amd/csrc/build; N=gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
for n in 65536 131072 262144; do
  for i in 1 2; do
    for lib in $B/lib_base.so $B/lib_wpe4.so $B/lib_rwin0.so $B/lib_rwin0w4.so; do
      AB_N=$n ST_LIB=$lib AB_LABEL="$(basename $lib) n=$n" timeout -k 10 120 python tools/ab_rollout.py 100 10 || exit 1
    done
  done
done | tee gpurun_out/ab_ro6.txt
