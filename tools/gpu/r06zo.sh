# r06zo: the parse kernel's length-byte stores: lens aligned to 16 (a16) or 128 (a128) bytes per block, the flush after the ring refill request (a16l), non-temporal stores (a16nt); cur = the tree
export TMPDIR=/tmp
O=gpurun_out/r06zo
mkdir -p $O
kt() { v=$1; kinds=$2; n=$3
  cd /tmp && KINDS=$kinds LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so SEED=2026 NBLK=$n DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$v -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/kt_${v}_$kinds.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_${v}_$kinds.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_$v -name "kt_kernel_stats.csv" | head -1)
  echo "== $v $kinds $(grep "$kinds rows" $O/kt_${v}_$kinds.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    for k in ("rows_parse", "rows_exec", "decompress_kernel<false, true>"):
        if k in n:
            print(f"   {k:12s} avg {float(r['AverageNs'])/1e6:8.3f} ms  n {r['Calls']}")
PY
  rm -rf $O/kt_$v
}
kt cur silesia 1048576 && kt a16 silesia 1048576 && kt a128 silesia 1048576 && kt a16l silesia 1048576 && kt a16nt silesia 1048576 && kt cur silesia 1048576 && kt a16 silesia 1048576 && kt a16l silesia 1048576
