#!/bin/bash
# HBM traffic of the decoder on the bench workload: separate rocprofv3 --pmc
# passes over `bench.py` (one counter group each), then tools/pmc_report.py
# writes profiles/pmc_decompress.json.  usage: tools/pmc_bench.sh OUTDIR
set -e
OUT=$(realpath -m "$1")
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu --no-compress --e2e-blocks 0 --frame-gib 0 --random-blocks 131072 --c5-total 0 --c1-blocks 0"
# the decoder's kernels: the row decoder's parse, execution and finisher
KRX=${KRX:-"rows_parse_kernel|rows_exec_kernel|decompress_kernel<false, true>"}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 420 rocprofv3 --kernel-include-regex "$KRX" --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$REPO/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
  echo "pass $i done: $grp"
done <<GROUPS
FETCH_SIZE
WRITE_SIZE
${PMC_QUICK:+}$( [ -z "$PMC_QUICK" ] && printf '%s\n%s' "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum" || true )
GROUPS
python3 "$REPO/tools/pmc_report.py" "$OUT" "$OUT/pmc_decompress.json" 1048576 4096 "${CAL:-}" > "$OUT/report.json"
