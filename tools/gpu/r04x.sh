# r04x: lone-block compress stages its block in 4 KiB chunks (waves 1-3) while wave 0 parses; A/B against the previous commit on the same box
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_codec.py -m gpu -x -q -k "single or solo" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_new_$i.log 2>&1 && LZ4M_LIB=tools/_abv/prev/_lz4m.so timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_prev_$i.log 2>&1
echo "== new $i"; head -2 $O/probe_c1_new_$i.log | tail -1; echo "== prev $i"; head -2 $O/probe_c1_prev_$i.log | tail -1
done
LZ4M_LIB=tools/_abv/wts/_lz4m.so timeout -k 10 120 python3 -u tools/probe_wts.py > $O/probe_wts.log 2>&1; cat $O/probe_wts.log
