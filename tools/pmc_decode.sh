#!/bin/bash
# PMC passes over the batched decoder (one counter group per rocprofv3 run).
# usage: tools/pmc_decode.sh OUTDIR [kernel-regex]   (env: NBLK, KINDS)
set -e
OUT=$(realpath -m "$1"); RX=${2:-decompress}
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export NBLK=${NBLK:-262144} KINDS=${KINDS:-silesia} REPS=1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$REPO/tools/prof_decode.py" > "$OUT/p$i.log" 2>&1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INST_LEVEL_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_BUSY_avr
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA
GROUPS
