# r06p: SQ counters of the round-6 rows parse (two counter groups, 262 144
# blocks of the bench's data), and its go-lane threshold at 32 / 40 / 48
# (kernel traces of the 1 M-block probe on the bench's blocks, seed 2026)
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
GA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
GB="SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
i=0
for g in "$GA" "$GB"; do i=$((i+1))
  cd /tmp && SEED=2026 NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex rows_parse --pmc $g -d $GRAFT_REPO_ROOT/$O/sq/p$i -o p$i --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/sq_p$i.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/sq_p$i.log; exit 1; }
  cd $GRAFT_REPO_ROOT
done
for d in $O/sq/p1 $O/sq/p2; do f=$(find $d -name "*counter_collection.csv" | head -1); mv $f $d/$(basename $d)_counter_collection.csv 2>/dev/null || true; done
python3 tools/pmc_sum.py $O/sq rows_parse > $O/sq_parse.txt && cat $O/sq_parse.txt
kt() { v=$1; L=""; [ $v != head ] && L=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so
  cd /tmp && LZ4M_LIB=$L SEED=2026 NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$v -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/kt_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_$v -name "kt_kernel_stats.csv" | head -1)
  echo "== $v $(grep 'silesia rows' $O/kt_$v.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    for k in ("rows_parse", "rows_exec"):
        if k in n:
            print(f"   {k:12s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
  rm -rf $O/kt_$v
}
kt head && kt ma32 && kt ma48 && kt head && kt ma32 && kt ma48
