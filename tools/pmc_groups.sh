#!/bin/bash
# tools/pmc_groups.sh OUTDIR KERNEL_REGEX GROUPFILE script.py [args]: one
# rocprofv3 --pmc pass per line of GROUPFILE over `python3 script.py args`.
set -e
OUT=$(realpath -m "$1"); RX=$2; GF=$(realpath "$3"); SCRIPT=$(realpath "$4"); shift 4
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$SCRIPT" "$@" > "$OUT/p$i.log" 2>&1
  echo "pass $i done: $grp"
done < "$GF"
