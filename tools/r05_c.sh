#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05c
B=gym-simpletetris_amd/csrc/build
timeout -k 10 120 python tools/region_probe.py > gpurun_out/r05c/region_probe_kernarg1.jsonl || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python tools/region_probe.py > gpurun_out/r05c/region_probe_kernarg0.jsonl || exit 1
ST_LIB=$R/$B/lib_ablation.so AB_BITS="0 65536 131072 32768 0" TAG=r05c_split2 EXTRA="--steps 2000 --warmup 100" \
  timeout -k 10 300 bash tools/ablate.sh || exit 1
