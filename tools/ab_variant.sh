#!/bin/bash
# tools/ab_variant.sh NAME "EXTRA FLAGS": build the C-ABI library with extra
# defines into tools/_abv/NAME/_lz4m.so (A/B timing runs via LZ4M_LIB).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/_abv/$1" /tmp/abobj
make -s -C "$R/python-lz4_amd/csrc" OBJDIR="/tmp/abobj/$1" OUT="$R/tools/_abv/$1/_lz4m.so" \
     FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2"
grep -A12 "rows_exec" "/tmp/abobj/$1/lz4m_rows.res" | grep -E "VGPRs:|Occupancy" | sed "s/^/$1: /"
