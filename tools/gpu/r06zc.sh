# r06zc: decoder tests of the tree (whole-literal blocks in the parse kernel,
# the slow path's one-step far copies, the block order); kernel traces of
# HEAD (base), + whole-literal blocks (wl), + slow path (wlx), + block order
# (ord = the tree), alternating
export TMPDIR=/tmp
O=gpurun_out/r06zc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame or literal" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -n 1 $O/dec_tests.log
kt() { v=$1
  cd /tmp && LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so SEED=2026 NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$v -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/kt_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_$v -name "kt_kernel_stats.csv" | head -1)
  echo "== $v $(grep 'silesia rows' $O/kt_$v.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    for k in ("rows_order", "rows_parse", "rows_exec", "decompress_kernel<false, true>"):
        if k in n:
            print(f"   {k:12s} avg {float(r['AverageNs'])/1e6:8.3f} ms  n {r['Calls']}")
PY
  rm -rf $O/kt_$v
}
kt base && kt wl && kt wlx && kt ord && kt base && kt ord && kt wlx
