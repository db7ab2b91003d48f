# r03e: parse-refill A/B, phase split, SQ counters of the decoder kernels
# (HEAD vs the round-2 code paths), counter calibration and decoder traffic
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/pc/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "decompress" > $O/tests_pc.log 2>&1 || { tail -30 $O/tests_pc.log; exit 1; }
for V in default pc; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  find $O/kt_$V -type f ! -name "*kernel_stats.csv" -delete
done
LZ4M_LIB=$PWD/tools/_prof/_lz4m_rprof.so NB=262144 timeout -k 10 200 python3 -u tools/prof_rows.py > $O/rows_phases.log 2>&1 || exit $?
for V in default c0; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=262144 REPS=1 timeout -k 10 400 bash tools/pmc_groups.sh $O/sq_$V "rows_exec_kernel|rows_parse_kernel" tools/pmc/sq_exec.txt tools/probe_rows.py > $O/sq_$V.log 2>&1 || exit $?
  find $O/sq_$V -type f ! -name "*counter_collection.csv" -delete
done
timeout -k 10 300 bash tools/pmc_cal.sh $O/cal > $O/cal.log 2>&1; echo cal=$?
find $O/cal -type f ! -name "*counter_collection.csv" ! -name "*.json" ! -name "*.log" -delete
CAL=$PWD/$O/cal/calibration.json timeout -k 10 900 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1; echo pmc=$?
find $O/pmc -type f ! -name "*counter_collection.csv" ! -name "*.json" -delete
echo "=== summary"
tail -1 $O/tests_pc.log
for V in default pc; do echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"; find $O/kt_$V -name "*kernel_stats.csv" -exec grep -h -E "rows_parse|rows_exec|decompress_kernel<false, true>" {} + | cut -d, -f1-5; done
tail -13 $O/rows_phases.log
python3 - <<'PY'
import csv, glob, collections
for v in ("default", "c0"):
    c = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/r03e/sq_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rows_exec" in r["Kernel_Name"]:
                c[r["Counter_Name"]] += float(r["Counter_Value"])
    print(v, {k: f"{x:.3e}" for k, x in sorted(c.items())})
PY
head -c 1500 $O/pmc/pmc_decompress.json
