# r06h: SQ counters of the final row executor (262 144 blocks; r06e's pass
# for HEAD = the round-5 code) and of the parallel-parse compressor
# (131 072 silesia-like blocks), two counter groups each
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
GA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
GB="SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
pass() { name=$1; rx=$2; grp=$3; shift 3
  cd /tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-include-regex "$rx" --pmc $grp -d $GRAFT_REPO_ROOT/$O/$name -o p1 --output-format csv -- python3 -u "$SCRIPT" > $GRAFT_REPO_ROOT/$O/$name.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/$name.log; exit 1; }
  cd $GRAFT_REPO_ROOT; }
SCRIPT=$GRAFT_REPO_ROOT/tools/probe_rows.py
pass exec_a rows_exec "$GA" NBLK=262144 DECS=rows REPS=1
pass exec_b rows_exec "$GB" NBLK=262144 DECS=rows REPS=1
SCRIPT=$GRAFT_REPO_ROOT/tools/prof_compress.py
pass pc_a pcompress_kernel "$GA" NBLK=131072 KINDS=silesia MODES=parallel REPS=1
pass pc_b pcompress_kernel "$GB" NBLK=131072 KINDS=silesia MODES=parallel REPS=1
for k in exec pc; do
  mkdir -p $O/$k; cp -r $O/${k}_a $O/$k/p1; cp -r $O/${k}_b $O/$k/p2
  f=$(find $O/$k/p2 -name "*counter_collection.csv" | head -1); mv $f $O/$k/p2/p2_counter_collection.csv 2>/dev/null || true
  rx=rows_exec; [ $k = pc ] && rx=pcompress_kernel
  python3 tools/pmc_sum.py $O/$k "$rx" > $O/sq_$k.txt; echo "-- $k"; cat $O/sq_$k.txt
done
tail -3 $O/pc_a.log
