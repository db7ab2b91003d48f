# r06zi: the finisher's lane copies end with one exact 16-byte put instead of
# byte loops (fin = the tree) vs sync3 (HEAD): decoder tests, kernel traces;
# then a plain copy beside the row decoder (tools/probe_concurrent.py)
export TMPDIR=/tmp
O=gpurun_out/r06zi
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame or literal or dict or single" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -n 1 $O/dec_tests.log
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
kt sync3 silesia 1048576 && kt fin silesia 1048576 && kt sync3 silesia 1048576 && kt fin silesia 1048576
timeout -k 10 300 python3 -u tools/probe_concurrent.py > $O/concurrent.log 2>&1 || { tail -5 $O/concurrent.log; exit 1; }
cat $O/concurrent.log
