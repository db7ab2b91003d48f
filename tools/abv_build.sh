#!/bin/bash
# Dev: an A/B or diagnostic variant of the C-ABI library that travels to the
# GPU box (tools/_abv is git-ignored, not gpurun-ignored):
#   tools/abv_build.sh NAME "-DMACRO=..."  ->  tools/_abv/NAME/_lz4m.so (LZ4M_LIB=...)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/_abv/$1"
make -s -C "$R/python-lz4_amd/csrc" OBJDIR="$R/tools/_abv/$1/obj" OUT="$R/tools/_abv/$1/_lz4m.so" \
     FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2" 2>&1 | grep -E "error" -A3 || true
rm -f "$R/tools/_abv/$1/obj/"*.o
grep -A9 "res_exec_kernel" "$R/tools/_abv/$1/obj/lz4m_resident.res" | grep -E "VGPRs:|Occupancy|LDS Size|Scratch" | sed "s/^/$1 /"
