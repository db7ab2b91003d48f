# r04ai: pooled packing / unpacking of compress_many / decompress_many: block API tests + config-1 batched numbers
export TMPDIR=/tmp
O=gpurun_out/r04ai
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q -k "many or block" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-compress --e2e-blocks 0 --frame-gib 0 --c5-total 0 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c1.json')); print(d['extra'].get('config1'))"
