# r03d: GPU suite on the new default (aligned LDS), A/B with per-kernel times,
# bench and its rocprofv3 kernel stats
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
for V in default a2 a1c a1p c0; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  find $O/kt_$V -type f ! -name "*kernel_stats.csv" -delete
done
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_bench -o kt -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/bench_rocprof.err; rc=$?
find $O/kt_bench -type f ! -name "*kernel_stats.csv" -delete
echo "=== summary"
tail -1 $O/gpu_tests.log
for V in default a2 a1c a1p c0; do echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"; find $O/kt_$V -name "*kernel_stats.csv" -exec grep -h -E "rows_parse|rows_exec|decompress_kernel<false, true>" {} + | cut -d, -f1-5; done
head -c 700 $O/bench.json; echo
exit $rc
