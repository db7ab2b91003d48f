# r06zw: the parse's length bytes stored 32 at a time (a full 16-byte piece
# held in registers until the next: l32) against the tree (cur): decoder tests
# on l32, kernel traces alternating
export TMPDIR=/tmp
O=gpurun_out/r06zw
mkdir -p $O
LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/l32/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame or literal or long or unaligned" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_l32.log 2>&1 || { tail -30 $O/dec_tests_l32.log; exit 1; }
tail -n 1 $O/dec_tests_l32.log
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
kt cur silesia 1048576 && kt l32 silesia 1048576 && kt cur silesia 1048576 && kt l32 silesia 1048576
