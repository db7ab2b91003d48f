# r06j: is the row executor bound by its far-source line fills?  nofar (every
# far read aimed at the block start: wrong output, same instructions) against
# HEAD, and deeper histories at 5 waves per SIMD (1152 / 1280 B, keep 640 / 768)
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
for v in h1280 h1152; do
LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_$v.log 2>&1 || { tail -30 $O/dec_tests_$v.log; exit 1; }
tail -1 $O/dec_tests_$v.log
done
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head
run nofar LZ4M_LIB=$PWD/tools/_abv/nofar/_lz4m.so
run h1152 LZ4M_LIB=$PWD/tools/_abv/h1152/_lz4m.so
run h1280 LZ4M_LIB=$PWD/tools/_abv/h1280/_lz4m.so
run head2
run nofar2 LZ4M_LIB=$PWD/tools/_abv/nofar/_lz4m.so
run h1280b LZ4M_LIB=$PWD/tools/_abv/h1280/_lz4m.so
for v in nofar h1280; do
  cd /tmp && LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex rows_exec --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $GRAFT_REPO_ROOT/$O/pmc_$v/p1 -o p1 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/pmc_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/pmc_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT && python3 tools/pmc_sum.py $O/pmc_$v rows_exec > $O/pmc_$v.txt && echo "-- $v" && cat $O/pmc_$v.txt
done
