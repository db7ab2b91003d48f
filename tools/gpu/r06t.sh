# r06t: rows parse with the next step's token read as soon as this step's
# length is known (TOKAHEAD) -- decoder suites, then kernel traces of the
# 1 M-block probe on the bench's blocks, alternating with the same tree without it
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/ptok/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_ptok.log 2>&1 || { tail -30 $O/dec_tests_ptok.log; exit 1; }
tail -n 1 $O/dec_tests_ptok.log
kt() { v=$1
  cd /tmp && LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so SEED=2026 NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$v -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/kt_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_$v.log; exit 1; }
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
kt pbase2 && kt ptok && kt pbase2 && kt ptok
