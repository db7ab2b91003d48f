# r06zz: upper bound of dword-aligned far-source loads -- the executor's two
# far-source pieces requested at s0 & ~3 (wrong bytes, same control flow:
# timing only, fa) against the tree (cur); kernel traces alternating
export TMPDIR=/tmp
O=gpurun_out/r06zz
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
kt cur silesia 1048576 && kt fa silesia 1048576 && kt cur silesia 1048576 && kt fa silesia 1048576
