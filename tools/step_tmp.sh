#!/bin/bash
# dev: parallel-parse compressor A/B (previous / one packed prefix scan), two rounds each
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in pcf pch; do
    echo "== $v round $r"
    LZ4M_LIB=tools/_ab/$v/_lz4m.so NB=131072 KINDS=silesia,text timeout -k 10 180 python3 -u tools/probe_pc.py || exit 1
  done
done
