# r03h: executor with the literal bytes staged in LDS, no second far prefetch (fewer VGPRs)
# at 4 and 5 waves per SIMD (1 KiB history), against the default
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
for V in x4 x5; do
  LZ4M_LIB=$PWD/tools/_abv/$V/_lz4m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "decompress and rows" > $O/tests_$V.log 2>&1 || { tail -30 $O/tests_$V.log; exit 1; }
done
for V in default x4 x5; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  find $O/kt_$V -type f ! -name "*kernel_stats.csv" -delete
done
echo "=== summary"
for V in x4 x5; do tail -1 $O/tests_$V.log; done
for V in default x4 x5; do echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"; python3 - $O/kt_$V <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for k in ("rows_parse", "rows_exec", "decompress_kernel<false, true>"):
            if k in n: print(f"   {k:32s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
done
