# r05v: the offset's dword pair by a select tree (LZ4M_ROWS_OFFTREE, register selects only): the
# rows decoder suites first (short limit), then A/B at 1 M blocks
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "rows" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/rows_tests.log 2>&1 || { tail -30 $O/rows_tests.log; exit 1; }
tail -1 $O/rows_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or auto or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run tree1
run tree0 LZ4M_LIB=$PWD/tools/_abv/tree0/_lz4m.so
run tree1b
run tree0b LZ4M_LIB=$PWD/tools/_abv/tree0/_lz4m.so
