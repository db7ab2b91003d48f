# r06zs: what the parallel-parse compressor's byte-parallel output stores cost
# (pcns: the stores skipped, wrong output on purpose, timing only) against the tree
export TMPDIR=/tmp
O=gpurun_out/r06zs
mkdir -p $O
kt() { v=$1
  cd /tmp && NB=262144 LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$v -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_pc.py > $GRAFT_REPO_ROOT/$O/kt_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_$v -name "kt_kernel_stats.csv" | head -1)
  echo "== $v $(grep 'silesia:' $O/kt_$v.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "pcompress_kernel" in n:
        print(f"   {n.split('(')[0][:50]:50s} avg {float(r['AverageNs'])/1e6:8.3f} ms  n {r['Calls']}")
PY
  rm -rf $O/kt_$v
}
kt cur && kt pcns && kt cur && kt pcns
