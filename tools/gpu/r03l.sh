# r03l: LDS-staged lone-block kernels for the single-call API
# (lz4m_compress_solo, lz4m_decompress_solo) -- the single-call parity tests,
# the block API tests, then the per-call probe and its kernel statistics
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_capi.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
timeout -k 10 300 python3 -u tools/probe_c1.py > $O/probe_c1.log 2>&1 || { tail -20 $O/probe_c1.log; exit 1; }
(cd /tmp && N=200 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/probe_c1.py > $GRAFT_REPO_ROOT/$O/probe_c1_rocprof.log 2>&1) || exit $?
find $O/kt -type f ! -name "*kernel_stats.csv" -delete
echo "=== summary"
grep -E "passed|failed" $O/tests.log | tail -2
grep "us" $O/probe_c1.log
python3 - $O/kt <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
