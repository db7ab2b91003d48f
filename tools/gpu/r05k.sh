# r05k: perm-based LDS puts / dword-aligned reads (LZ4M_LDS_PERM) -- decoder suites, A/B at 1 M
# blocks; then the default bench under rocprofv3 kernel-trace stats
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto or hist or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -2 $O/dec_tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head
run perm0 LZ4M_LIB=$PWD/tools/_abv/perm0/_lz4m.so
run xp0 LZ4M_LIB=$PWD/tools/_abv/xp0/_lz4m.so
run head2
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.log || { tail -20 $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
cat $GRAFT_REPO_ROOT/$O/bench_prof.json | head -c 600
