# r06k: deeper row histories at 5 waves per SIMD (LDS-limited at 1392 B):
# keep / room splits, decoder suites for each, 1 M-block probes twice
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
for v in h1392 h1392k h1280k; do
LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_$v.log 2>&1 || { tail -30 $O/dec_tests_$v.log; exit 1; }
tail -n 1 $O/dec_tests_$v.log
done
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
for k in 1 2; do
run head$k
for v in h1280 h1280k h1392 h1392k; do run $v$k LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
done
