# r06d: the speculative token-chain parse (LZ4M_PARSE_SPEC=2 / 4 sequences per
# fast step): decoder suites through spec4, 1 M-block probes, and rocprofv3
# kernel traces (262 144 blocks) of HEAD and spec4 for the parse kernel alone
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/spec4/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_spec4.log 2>&1 || { tail -30 $O/dec_tests_spec4.log; exit 1; }
tail -1 $O/dec_tests_spec4.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head
run spec4 LZ4M_LIB=$PWD/tools/_abv/spec4/_lz4m.so
run spec2 LZ4M_LIB=$PWD/tools/_abv/spec2/_lz4m.so
run head2
run spec4b LZ4M_LIB=$PWD/tools/_abv/spec4/_lz4m.so
for v in head spec4; do
  L=""; [ $v = spec4 ] && L=$GRAFT_REPO_ROOT/tools/_abv/spec4/_lz4m.so
  cd /tmp && LZ4M_LIB=$L NBLK=262144 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o k --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); grep -E "rows_parse|rows_exec|decompress_kernel" $f | cut -d, -f1-8
done
