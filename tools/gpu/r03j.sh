# r03j: GPU suite at HEAD (mirror-free parse ring, prefetching XXH32 lane
# loop); A/B of the history split (kept bytes / room per round at 1 KiB);
# full bench (config 1 per call, config 5 consumer); kernel trace of config 1
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
for V in k640 k768 k384; do
  LZ4M_LIB=$PWD/tools/_abv/$V/_lz4m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "decompress and rows" > $O/tests_$V.log 2>&1 || { tail -30 $O/tests_$V.log; exit 1; }
done
for V in default k640 k768 k384; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  find $O/kt_$V -type f ! -name "*kernel_stats.csv" -delete
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c1 -o kt -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-compress --e2e-blocks 0 --frame-gib 0 --random-blocks 0 --c5-total 0 --c1-blocks 300 > $O/c1.json 2> $O/c1.err || exit $?
find $O/kt_c1 -type f ! -name "*kernel_stats.csv" -delete
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "=== summary"
tail -1 $O/gpu_tests.log
for V in k640 k768 k384; do tail -1 $O/tests_$V.log; done
for V in default k640 k768 k384; do echo "$V: $(grep -o '"silesia/rows": {[^}]*}' $O/probe_$V.log)"; python3 - $O/kt_$V <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for k in ("rows_parse", "rows_exec", "decompress_kernel<false, true>"):
            if k in n: print(f"   {k:32s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
done
python3 - $O/kt_c1 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"c1 {r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
python3 -c "
import json; d = json.load(open('$O/bench.json')); e = d['extra']
print('value', d['value'], d['roofline'])
print('c1', {k: e['config1'][k] for k in ('per_call_compress_us', 'per_call_decompress_us', 'batched_roundtrip_gib_s')})
print('c5', e['config5']['weak'])
print('frame4m', {k: e['frame4m'][k] for k in ('compress_frame_gib_s', 'decompress_frame_gib_s')})"
