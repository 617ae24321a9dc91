#!/bin/bash
# Round 5: the hot-row + cold-record state layout -- GPU suite, A/B against
# the round-5 start layout (lib_base.so), PMC traffic of both.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05g
B=$R/gym-simpletetris_amd/csrc/build
NEW=$R/gym-simpletetris_amd/gym_simpletetris_amd/libsimpletetris.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_base.so $NEW; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05g/ab_layout.txt || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in $B/lib_base.so $NEW; do
  n=$(basename $lib .so)
  ST_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r05g/pmcf_$n -o p -- python3 $R/tools/ab_step.py 600 > /dev/null 2>&1 || exit 1
  ST_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r05g/pmcw_$n -o p -- python3 $R/tools/ab_step.py 600 > /dev/null 2>&1 || exit 1
  (cd $R && python3 tools/pmc_quick.py gpurun_out/r05g/pmcf_$n gpurun_out/r05g/pmcw_$n > gpurun_out/r05g/pmc_$n.txt) || exit 1
done
find $R/gpurun_out/r05g -name "*.csv" ! -name "*counter_collection.csv" -delete
