# r04am: final tree -- GPU suite, smoke(), bench (default flags), then the
# rocprofv3 kernel statistics of the same bench command
export TMPDIR=/tmp
O=gpurun_out/r04am
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['roofline'])
print(d['extra'].get('config1'))
print(d['compress'].get('compress_exact_gib_s'), d['extra']['frame4m'])"
