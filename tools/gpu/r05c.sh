# r05c: row executor with loads in flight across rounds (parse ahead after the passes, two far
# pieces, length bytes carried as prefix sums), parse run cap: decoder tests + 1 M-block A/B
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decomp or decode or rows or roundtrip or round_trip" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run base0 LZ4M_LIB=$PWD/tools/_abv/base/_lz4m.so
run new0
run nocap LZ4M_LIB=$PWD/tools/_abv/nocap/_lz4m.so
run new1
run base1 LZ4M_LIB=$PWD/tools/_abv/base/_lz4m.so
