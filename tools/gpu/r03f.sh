# r03f: A/B of history size, skipped empty masked ORs, cooperative parse
# refills; FETCH/WRITE_SIZE of the decoder kernels per variant
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
for V in h3k h4k sk; do
  LZ4M_LIB=$PWD/tools/_abv/$V/_lz4m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "decompress and rows" > $O/tests_$V.log 2>&1 || { tail -30 $O/tests_$V.log; exit 1; }
done
for V in default sk pc h1k h3k h4k; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  find $O/kt_$V -type f ! -name "*kernel_stats.csv" -delete
done
for V in default h3k h4k pc; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && LZ4M_LIB=$L DECS=rows NBLK=262144 REPS=1 timeout -s KILL 180 rocprofv3 --kernel-include-regex "rows_exec|rows_parse|decompress_kernel" --pmc $C -d $GRAFT_REPO_ROOT/$O/pmc_${V}_$C -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/pmc_${V}_$C.log 2>&1) || exit $?
  done
done
echo "=== summary"
for V in h3k h4k sk; do tail -1 $O/tests_$V.log; done
for V in default sk pc h1k h3k h4k; do echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"; python3 - $O/kt_$V <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for k in ("rows_parse", "rows_exec", "decompress_kernel<false, true>"):
            if k in n: print(f"   {k:32s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
done
python3 - <<'PY'
import csv, glob
for v in ("default", "h3k", "h4k", "pc"):
    out = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"gpurun_out/r03f/pmc_{v}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].split("::")[-1][:20] + "." + c[0]
                out[k] = out.get(k, 0) + float(r["Counter_Value"]) * 1024 / 2 / 1e9   # 2 launches: GB per launch
    print(v, {k: round(x, 2) for k, x in sorted(out.items())})
PY
