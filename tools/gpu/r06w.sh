# r06w: row executor workgroups of 5 waves (20 rows; 4 workgroups x 5 = 20
# waves per CU as before) with the LDS that frees spent on 1376-byte histories
# (e320) or not (e320h); decoder suites on e320; kernel traces on the bench's blocks
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/e320/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_e320.log 2>&1 || { tail -30 $O/dec_tests_e320.log; exit 1; }
tail -n 1 $O/dec_tests_e320.log
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
kt head && kt e320 && kt e320h && kt head && kt e320 && kt e320h
