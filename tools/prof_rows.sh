#!/bin/bash
# Diagnostic build of the C-ABI library with the row decoder's phase
# counters (-DLZ4M_ROWS_PROF) into tools/_prof/_lz4m_rprof.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/_prof"
make -s -C "$R/python-lz4_amd/csrc" OBJDIR="$R/tools/_prof/robj" OUT="$R/tools/_prof/_lz4m_rprof.so" \
     FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -DLZ4M_ROWS_PROF $EXTRA"
