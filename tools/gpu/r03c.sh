# r03c: LDS alignment micro-benchmark; parity of the aligned-LDS variant
# (rows exec + parse + hist); decoder A/B with per-kernel times; phase split
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 120 tools/micro/lds_align > $O/lds_align.log 2>&1 || exit $?
LZ4M_LIB=$PWD/tools/_abv/alp/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "decompress" > $O/tests_alp.log 2>&1 || { tail -30 $O/tests_alp.log; exit 1; }
tail -1 $O/tests_alp.log
for V in default alp al al3 n1 p0 c0; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  find $O/kt_$V -type f ! -name "*kernel_stats.csv" -delete
  echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"
done
for V in default alp; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=hist NBLK=16384 REPS=3 timeout -k 10 200 python3 tools/probe_rows.py > $O/probe_hist_$V.log 2>&1 || exit $?
done
LZ4M_LIB=$PWD/tools/_prof/_lz4m_rprof.so NB=262144 timeout -k 10 200 python3 -u tools/prof_rows.py > $O/rows_phases.log 2>&1 || exit $?
echo "=== summary"
tail -1 $O/tests_alp.log
for V in default alp al al3 n1 p0 c0; do echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"; find $O/kt_$V -name "*kernel_stats.csv" -exec grep -h -E "rows_parse|rows_exec|decompress_kernel" {} + | cut -d, -f1-4; done
for V in default alp; do echo "hist $V: $(grep -o '"silesia/hist": {[^}]*}' $O/probe_hist_$V.log)"; done
grep -E "mskor|misalign\": 0|misalign\": 1," $O/lds_align.log | cut -c1-110
tail -13 $O/rows_phases.log
