#!/bin/bash
# GPU test suite on the box: tools/gpu/suite.sh OUTDIR [pytest args...]
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/suite}; shift
mkdir -p "$out"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider "$@" > "$out/gputest.log" 2>&1
rc=$?
tail -5 "$out/gputest.log"
exit $rc
