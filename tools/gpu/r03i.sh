# r03i: HEAD (5-wave executor) -- GPU suite, bench and its rocprofv3 kernel
# stats, decoder traffic (calibrated method), rows_exec SQ counters; A/B of the
# mirror-free parse ring (nm); random-block dispatch write/fetch check
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/nm/_lz4m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "decompress and rows" > $O/tests_nm.log 2>&1 || { tail -30 $O/tests_nm.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
for V in default nm; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  find $O/kt_$V -type f ! -name "*kernel_stats.csv" -delete
done
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_bench -o kt -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/bench_rocprof.err || exit $?
find $O/kt_bench -type f ! -name "*kernel_stats.csv" -delete
DECS=rows NBLK=262144 REPS=1 timeout -k 10 400 bash tools/pmc_groups.sh $O/sq_default "rows_exec_kernel|rows_parse_kernel" tools/pmc/sq_exec.txt tools/probe_rows.py > $O/sq_default.log 2>&1 || exit $?
find $O/sq_default -type f ! -name "*counter_collection.csv" -delete
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && KINDS=random DECS=rows NBLK=131072 REPS=1 timeout -s KILL 180 rocprofv3 --kernel-include-regex "rows_exec|rows_parse|decompress_kernel" --pmc $C -d $GRAFT_REPO_ROOT/$O/rand_$C -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/rand_$C.log 2>&1) || exit $?
done
CAL=$PWD/profiles/r03/r03e_traffic_calibration.json timeout -k 10 900 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1 || exit $?
find $O/pmc -type f ! -name "*counter_collection.csv" ! -name "*.json" -delete
echo "=== summary"
tail -1 $O/tests_nm.log
tail -1 $O/gpu_tests.log
for V in default nm; do echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"; python3 - $O/kt_$V <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for k in ("rows_parse", "rows_exec", "decompress_kernel<false, true>"):
            if k in n: print(f"   {k:32s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
done
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(float)
for f in glob.glob("gpurun_out/r03i/sq_default/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rows_exec" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"])
print("sq", {k: f"{x:.4e}" for k, x in sorted(c.items())})
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/r03i/rand_{C}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"].split("(")[0][-24:], r["Dispatch_Id"])] += float(r["Counter_Value"]) * 1024
    print("random", C, {f"{k[0]}#{k[1]}": round(v / 1e9, 3) for k, v in sorted(per.items(), key=lambda z: int(z[0][1]))})
PY
head -c 1200 $O/pmc/pmc_decompress.json; echo
head -c 900 $O/bench.json; echo
