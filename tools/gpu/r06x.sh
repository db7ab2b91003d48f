# r06x: the executor flushing whole 128-byte lines only (each line written
# once; FLUSH128) -- decoder suites, kernel traces alternating with the same
# tree without it, and WRITE_SIZE / FETCH_SIZE of rows_exec for both
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/f128/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_f128.log 2>&1 || { tail -30 $O/dec_tests_f128.log; exit 1; }
tail -n 1 $O/dec_tests_f128.log
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
kt fbase && kt f128 && kt fbase && kt f128
for v in fbase f128; do for g in WRITE_SIZE FETCH_SIZE; do
  cd /tmp && LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so SEED=2026 NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex rows_exec --pmc $g -d $GRAFT_REPO_ROOT/$O/pmc_${v}_$g/p1 -o p1 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/pmc_${v}_$g.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/pmc_${v}_$g.log; exit 1; }
  cd $GRAFT_REPO_ROOT && echo "-- $v $g" && python3 tools/pmc_sum.py $O/pmc_${v}_$g rows_exec
done; done
