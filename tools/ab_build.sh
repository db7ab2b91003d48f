#!/bin/bash
# Dev: an A/B variant of the C-ABI library: tools/ab_build.sh NAME "-DMACRO=..."
# -> tools/_ab/NAME/_lz4m.so (load it with LZ4M_LIB=...).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/_ab/$1"
make -s -C "$R/python-lz4_amd/csrc" OBJDIR="$R/tools/_ab/$1/obj" OUT="$R/tools/_ab/$1/_lz4m.so" \
     FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2" 2>&1 | grep -v "stop' set but" | grep -v "^ *[0-9]* |" | grep -v "^ *|" || true
grep -A8 "rows_parse_kernel\|rows_exec_kernel" "$R/tools/_ab/$1/obj/lz4m_rows.res" | grep -E "VGPRs:|Occupancy|LDS Size" | sed "s/^/$1 /"
