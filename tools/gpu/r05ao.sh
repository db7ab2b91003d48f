# r05ao: VOP3 selects in asm with the two wait states before and after (the asm without them faulted in
# r05an): row decoder suites on the new build, then A/B at 1 M blocks against the plain ternaries (novop3)
export TMPDIR=/tmp
O=gpurun_out/r05ao
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "rows" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run vop3
run novop3 LZ4M_LIB=$PWD/tools/_abv/novop3/_lz4m.so
run vop3b
run novop3b LZ4M_LIB=$PWD/tools/_abv/novop3/_lz4m.so
