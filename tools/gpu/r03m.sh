# r03m: HEAD (lone-block single-call kernels) -- GPU suite, per-call probe (config 1 fixed costs), decoder
# traffic for HEAD's decoder (calibrated method) copied to
# profiles/pmc_decompress.json before the bench so roofline.traffic is filled,
# bench and its rocprofv3 kernel stats
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python3 -u tools/probe_c1.py > $O/probe_c1.log 2>&1 || { tail -20 $O/probe_c1.log; exit 1; }
CAL=$PWD/profiles/r03/r03e_traffic_calibration.json timeout -k 10 1200 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
find $O/pmc -type f ! -name "*counter_collection.csv" ! -name "*.json" -delete
cp $O/pmc/pmc_decompress.json profiles/pmc_decompress.json
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_bench -o kt -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/bench_rocprof.err || exit $?
find $O/kt_bench -type f ! -name "*kernel_stats.csv" -delete
echo "=== summary"
tail -1 $O/gpu_tests.log
cat $O/probe_c1.log | grep "us"
head -c 1500 $O/pmc/pmc_decompress.json; echo
head -c 900 $O/bench.json; echo
