# r05w: far sources read back from the lane's literal slot (LZ4M_ROWS_FARXS): the rows decoder
# suites with it (variant library), then A/B at 1 M blocks
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/farxs/_lz4m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "rows" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/rows_tests.log 2>&1 || { tail -30 $O/rows_tests.log; exit 1; }
tail -1 $O/rows_tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run farxs1 LZ4M_LIB=$PWD/tools/_abv/farxs/_lz4m.so
run farxs0 LZ4M_LIB=$PWD/tools/_abv/farxs0/_lz4m.so
run farxs1b LZ4M_LIB=$PWD/tools/_abv/farxs/_lz4m.so
run farxs0b LZ4M_LIB=$PWD/tools/_abv/farxs0/_lz4m.so
