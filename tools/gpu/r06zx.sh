# r06zx: SQ counters of the final row executor and rows parse (262 144 bench
# blocks, two launches; two counter groups each), for the next round
export TMPDIR=/tmp
O=gpurun_out/r06zx
mkdir -p $O
GA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
GB="SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
pass() { name=$1; rx=$2; grp=$3
  cd /tmp && SEED=2026 NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex "$rx" --pmc $grp -d $GRAFT_REPO_ROOT/$O/$name -o p1 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/$name.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/$name.log; exit 1; }
  cd $GRAFT_REPO_ROOT; }
pass exec_a rows_exec "$GA" && pass exec_b rows_exec "$GB" && pass parse_a rows_parse "$GA" && pass parse_b rows_parse "$GB"
for k in exec parse; do
  mkdir -p $O/$k; cp -r $O/${k}_a $O/$k/p1; cp -r $O/${k}_b $O/$k/p2
  f=$(find $O/$k/p2 -name "*counter_collection.csv" | head -1); mv $f $O/$k/p2/p2_counter_collection.csv 2>/dev/null || true
  rx=rows_exec; [ $k = parse ] && rx=rows_parse
  python3 tools/pmc_sum.py $O/$k "$rx" > $O/sq_$k.txt; echo "-- $k"; cat $O/sq_$k.txt
done
