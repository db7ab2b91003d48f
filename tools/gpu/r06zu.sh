# r06zu: the parallel-parse compressor at 19 instead of 20 waves per CU (256 B more LDS per workgroup, pcpad)
export TMPDIR=/tmp
O=gpurun_out/r06zu
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
kt cur && kt pcpad && kt cur && kt pcpad
