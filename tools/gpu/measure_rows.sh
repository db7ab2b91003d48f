#!/bin/bash
# Row decoder measurements on the box: tools/gpu/measure_rows.sh OUTDIR
#   probe.log   -- decode time at NBLK blocks (default 262 144), verified
#   kt/         -- rocprofv3 kernel trace + stats of the same run
#   phases.log  -- per-phase wave-cycle split (tools/_prof/_lz4m_rprof.so)
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/rows}
mkdir -p "$out"
nb=${NBLK:-262144}
DECS=${DECS:-rows} NBLK=$nb REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt" -o kt -- \
    python3 tools/probe_rows.py > "$out/probe.log" 2>&1 || exit $?
tail -2 "$out/probe.log"
if [ -f tools/_prof/_lz4m_rprof.so ] && [ -z "$NOPHASE" ]; then
    LZ4M_LIB=$PWD/tools/_prof/_lz4m_rprof.so NB=$nb timeout -k 10 240 python3 -u tools/prof_rows.py \
        > "$out/phases.log" 2>&1 || exit $?
    cat "$out/phases.log"
fi
