#!/bin/bash
# PMC passes over the parallel-parse compressor (one counter group per rocprofv3 run).
# usage: tools/pmc_pcompress.sh OUTDIR   (env: NB)
set -e
OUT=$(realpath -m "$1")
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export NB=${NB:-65536}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-include-regex pcompress --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$REPO/tools/probe_pc.py" > "$OUT/p$i.log" 2>&1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE
GROUPS
