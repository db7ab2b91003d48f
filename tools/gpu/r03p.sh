# r03p: final tree of the session -- GPU suite, smoke(), bench (config-1 line
# on the staged single-call path; roofline.traffic must still match)
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "=== summary"
tail -1 $O/gpu_tests.log
tail -1 $O/smoke.log
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['roofline'])
print(d['extra']['config1'])
print(d['compress']['compress_exact_gib_s'], d['extra']['frame4m']['decompress_frame_gib_s'])"
