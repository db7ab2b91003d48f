#!/bin/bash
# Traffic-counter calibration on known-bytes kernels (tools/micro/traffic_cal):
# one rocprofv3 --pmc pass per counter group, then tools/pmc_cal_report.py.
# usage: tools/pmc_cal.sh OUTDIR
set -e
OUT=$(realpath -m "$1")
REPO=$(cd "$(dirname "$0")/.." && pwd)
BIN="$REPO/tools/micro/traffic_cal"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$BIN" > "$OUT/plain.log"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- "$BIN" > "$OUT/p$i.log" 2>&1
  echo "cal pass $i done: $grp"
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum
GROUPS
python3 "$REPO/tools/pmc_cal_report.py" "$OUT" > "$OUT/calibration.json"
cat "$OUT/calibration.json"
