#!/bin/bash
# Dev helper: tools/gpu.sh CMDFILE [timeout] -- run gpurun with the command in
# CMDFILE; retry only infrastructure transients (nothing ran, nothing charged).
CMD=$(cat "$1"); T=${2:-900}
cd "$(dirname "$0")/.."
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > gpurun_out/call.log 2>&1
  rc=$?
  if grep -q "status=transient" gpurun_out/call.log; then
    echo "transient (attempt $i), retrying in 45s"; sleep 45; continue
  fi
  break
done
tail -4 gpurun_out/call.log
exit $rc
