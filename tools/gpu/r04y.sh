# r04y: rocprofv3 kernel statistics of the default bench command, then the
# decoder's PMC traffic passes (FETCH_SIZE / WRITE_SIZE) for roofline.traffic
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
R=$(pwd)
(cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py > $R/$O/bench_prof.json 2> $R/$O/bench_prof.err) || { tail -20 $O/bench_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats_bench.csv
PMC_QUICK=1 CAL=$R/profiles/traffic_calibration.json timeout -k 10 600 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cat $O/pmc/report.json | head -40
