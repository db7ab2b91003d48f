#!/bin/bash
# Round-end evidence: decoder HBM traffic (PMC passes, tools/pmc_bench.sh) and a
# rocprofv3 kernel-trace --stats run of the default bench command.
# usage: tools/prof_round.sh TAG   (writes gpurun_out/pmc_TAG, gpurun_out/stats_TAG)
REPO=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1
cd "$REPO"
bash tools/pmc_bench.sh gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.log 2>&1
echo "pmc rc=$?"; cat gpurun_out/pmc_$TAG.log | tail -5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/stats_$TAG" -o st --output-format csv -- python3 "$REPO/bench.py" > "$REPO/gpurun_out/stats_$TAG.json" 2> "$REPO/gpurun_out/stats_$TAG.err"
echo "stats rc=$?"; tail -c 600 "$REPO/gpurun_out/stats_$TAG.json"
