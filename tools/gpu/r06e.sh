# r06e: executor VALU cuts -- unsigned in-block offsets (u32), literals at parse
# time + OR puts + the first match put's selectors once per round (lop, lopu
# = lop + u32): decoder suites through lopu, 1 M-block probes, and one SQ
# counter pass over rows_exec (262 144 blocks) for HEAD and lopu
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/lopu/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests_lopu.log 2>&1 || { tail -30 $O/dec_tests_lopu.log; exit 1; }
tail -1 $O/dec_tests_lopu.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head
run u32 LZ4M_LIB=$PWD/tools/_abv/u32/_lz4m.so
run litnow LZ4M_LIB=$PWD/tools/_abv/litnow/_lz4m.so
run lop LZ4M_LIB=$PWD/tools/_abv/lop/_lz4m.so
run lopu LZ4M_LIB=$PWD/tools/_abv/lopu/_lz4m.so
run head2
run lopu2 LZ4M_LIB=$PWD/tools/_abv/lopu/_lz4m.so
for v in head lopu; do
  L=""; [ $v != head ] && L=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so
  cd /tmp && LZ4M_LIB=$L NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex rows_exec --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $GRAFT_REPO_ROOT/$O/pmc_$v/p1 -o p1 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/pmc_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/pmc_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT && python3 tools/pmc_sum.py $O/pmc_$v rows_exec > $O/pmc_$v.txt && echo "-- $v" && cat $O/pmc_$v.txt
done
