# r05q: the match offset read back from the literal's LDS slot (LZ4M_ROWS_OFFLDS) and 256-thread
# executor workgroups (LZ4M_ROWS_EWG=256): decoder suites, A/B at 1 M blocks
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head
run off0 LZ4M_LIB=$PWD/tools/_abv/off0/_lz4m.so
run ewg256 LZ4M_LIB=$PWD/tools/_abv/ewg256/_lz4m.so
run head2
