# r05d: parse kernel V2 (predicated two-step fast loop, ring stops without the general parse, one-extension
# general parse): decoder tests + 1 M-block A/B against V1 + kernel trace of both
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decomp or decode or rows or roundtrip or round_trip" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt -- python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run v2a
run v1 LZ4M_LIB=$PWD/tools/_abv/pv1/_lz4m.so
run v2b
