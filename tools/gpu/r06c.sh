# r06c: executor A/Bs -- ORPUT (history kept zero, puts as ds_or_b32), LITNOW
# (literals placed at parse time, no LDS literal slot), both: decoder suites
# through the combined build, then 1 M-block probes
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/orlit/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_orlit.log 2>&1 || { tail -30 $O/dec_tests_orlit.log; exit 1; }
tail -1 $O/dec_tests_orlit.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head
run orput LZ4M_LIB=$PWD/tools/_abv/orput/_lz4m.so
run litnow LZ4M_LIB=$PWD/tools/_abv/litnow/_lz4m.so
run orlit LZ4M_LIB=$PWD/tools/_abv/orlit/_lz4m.so
run head2
run orlit2 LZ4M_LIB=$PWD/tools/_abv/orlit/_lz4m.so
