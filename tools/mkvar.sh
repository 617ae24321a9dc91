#!/bin/bash
# usage: mkvar.sh <kernel source> <name> [extra defs]   -> build/lib_<name>.so
set -e
cd /root/repo/gym-simpletetris_amd/csrc
SRC=$1; V=$2; shift 2
mkdir -p build
cp "$SRC" build/var_$V.hip
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I/root/repo/include -I. "$@" -c build/var_$V.hip -o build/k_$V.o 2>&1 | grep -E "error" -A3 || true
[ -f build/st_capi.cpp.o ] || make -s
hipcc --offload-arch=gfx950 -shared -fPIC -o build/lib_$V.so build/k_$V.o build/st_capi.cpp.o 2>&1 | grep -v hip-link || true
ls -la build/lib_$V.so
