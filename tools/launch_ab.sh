#!/bin/bash
# A/B of the timed region's launch mode (hipGraph replay vs K eager ctypes
# launches) at the driver's short shape and the default long one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/launch_ab.jsonl
: > $out
for rep in 1 2 3; do
  for shape in "20 5" "4000 100"; do
    set -- $shape
    for mode in graph eager; do
      timeout -k 10 120 python bench.py --steps $1 --warmup $2 --launch $mode --no-extras --no-cpu-baseline \
        > gpurun_out/lab.json 2>> gpurun_out/launch_ab.err || exit 1
      python -c "
import json,sys; d=json.loads(open('gpurun_out/lab.json').read().strip().splitlines()[-1])
print(json.dumps({'mode':'$mode','K':$1,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernel_us':d['roofline']['kernel_us']}))" | tee -a $out
    done
  done
done
