#!/bin/bash
# tools/pmc_run.sh OUTDIR KERNEL_REGEX script.py [args]: one rocprofv3 --pmc
# pass per counter group over `python3 script.py args` (env passes through).
set -e
OUT=$(realpath -m "$1"); RX=$2; SCRIPT=$(realpath "$3"); shift 3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex "$RX" --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$SCRIPT" "$@" > "$OUT/p$i.log" 2>&1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG
GROUPS
