#!/bin/bash
# Round 5: cold-record store shapes -- A/B of the round-5 start layout
# (lib_base), the current build (lib_cur: masked 16-B + dword stores) and
# whole-sector rewrites (lib_full), with PMC traffic; full-sector parity.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r05l
B=$R/gym-simpletetris_amd/csrc/build
ST_LIB=$B/lib_full.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_horizon.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05l/pytest_full.log 2>&1 || exit 1
for i in 1 2 3; do
  for lib in $B/lib_base.so $B/lib_cur.so $B/lib_full.so; do
    echo "$(basename $lib) $(ST_LIB=$lib timeout -k 10 120 python tools/ab_step.py 2000)" >> gpurun_out/r05l/ab_layout.txt || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in $B/lib_base.so $B/lib_cur.so $B/lib_full.so; do
  n=$(basename $lib .so)
  ST_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r05l/pmcf_$n -o p -- python3 $R/tools/ab_step.py 600 > /dev/null 2>&1 || exit 1
  ST_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r05l/pmcw_$n -o p -- python3 $R/tools/ab_step.py 600 > /dev/null 2>&1 || exit 1
  (cd $R && python3 tools/pmc_quick.py gpurun_out/r05l/pmcf_$n gpurun_out/r05l/pmcw_$n > gpurun_out/r05l/pmc_$n.txt) || exit 1
done
find $R/gpurun_out/r05l -name "*.csv" ! -name "*counter_collection.csv" -delete
