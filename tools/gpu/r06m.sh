# r06m: rows parse fast loop with one condition per step for the going lanes
# (pgo: the stop reason found after the loop, SALU per step 33 -> 9), 2 / 4
# steps per exit test, the general parse from aligned dword pairs (GEN2);
# decoder suites on pgo4g; kernel traces of the 1 M-block probe
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
for v in pgo4g pgo; do
LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_$v.log 2>&1 || { tail -30 $O/dec_tests_$v.log; exit 1; }
tail -n 1 $O/dec_tests_$v.log
done
for v in pnew4 pgo pgo4 pgo4g pnew4g pgo4 pgo4g; do
  cd /tmp && LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$v -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/kt_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_$v -name "kt_kernel_stats.csv" | head -1)
  echo "== $v $(grep 'silesia rows' $O/kt_$v.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "rows_parse" in n:
        print(f"   parse calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
  rm -rf $O/kt_$v
done
