#!/bin/bash
# Dev helper: tools/gpu.sh CMDFILE [timeout] -- run gpurun with the command in
# CMDFILE; retry only infrastructure transients (nothing ran, nothing charged)
# and "no box free" (rc 3), backing off as gpurun asks.
CMD=$(cat "$1"); T=${2:-900}
cd "$(dirname "$0")/.."
for i in $(seq 1 25); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > gpurun_out/call.log 2>&1
  rc=$?
  if grep -q "status=transient" gpurun_out/call.log || [ $rc -eq 3 ]; then
    w=$(grep -o "retry in [0-9]*s" gpurun_out/call.log | grep -o "[0-9]*" | head -1)
    w=${w:-60}; [ "$w" -lt 45 ] && w=45
    echo "transient/no box (attempt $i, rc=$rc), retrying in ${w}s"; sleep "$w"; continue
  fi
  break
done
tail -4 gpurun_out/call.log
exit $rc
