# r05e: phase profiles (parse V2 / V1, executor), macro A/Bs at 1 M blocks, parse SQ counters V2,
# batched launch beside a single-call loop
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q -s -k "beside_single_call or many_threads" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "batched decode|passed|failed" $O/tests.log
LZ4M_LIB=$PWD/tools/_abv/rprof/_lz4m.so NB=262144 timeout -k 10 240 python3 -u tools/prof_rows.py > $O/phases_v2.log 2>&1 || { tail -5 $O/phases_v2.log; exit 1; }
cat $O/phases_v2.log
LZ4M_LIB=$PWD/tools/_abv/rprofv1/_lz4m.so NB=262144 timeout -k 10 240 python3 -u tools/prof_rows.py > $O/phases_v1.log 2>&1 || { tail -5 $O/phases_v1.log; exit 1; }
cat $O/phases_v1.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head0
for v in al2 pass1 minact48 minact32; do run $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
run head1
NBLK=262144 DECS=rows REPS=1 bash tools/pmc_groups.sh $O/pmc_parse rows_parse tools/pmc/sq_parse2.txt tools/probe_rows.py || exit 1
