# r05o: decoder A/Bs at 1 M blocks -- HEAD (put selector base by v_perm), unneeded put dwords
# skipped (LZ4M_LDS_SKIP), 256-thread executor workgroups (LZ4M_ROWS_EWG, tables shared by 4 waves)
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head
run skip1 LZ4M_LIB=$PWD/tools/_abv/skip1/_lz4m.so
run ewg256 LZ4M_LIB=$PWD/tools/_abv/ewg256/_lz4m.so
run head2
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "rows or auto" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
