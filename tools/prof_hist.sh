#!/bin/bash
# Diagnostic build of the C-ABI library with hist_decompress_kernel's phase
# counters (-DLZ4M_HIST_PROF) into tools/_prof/_lz4m_prof.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/_prof"
make -s -C "$R/python-lz4_amd/csrc" OBJDIR="$R/tools/_prof/obj" OUT="$R/tools/_prof/_lz4m_prof.so" \
     FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -DLZ4M_HIST_PROF"
