# r06zj: deeper row histories at lower occupancy now that the executor reads
# ~6 TB/s of far-source line fills: 1536 / 1792 B (4 workgroups per CU) and
# 2560 B (3 per CU) against 1280 B at 5 (sync3 = HEAD); kernel traces, alternating
export TMPDIR=/tmp
O=gpurun_out/r06zj
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
kt sync3 silesia 1048576 && kt h1536 silesia 1048576 && kt h1792 silesia 1048576 && kt h2560 silesia 1048576 && kt sync3 silesia 1048576 && kt h1792 silesia 1048576
