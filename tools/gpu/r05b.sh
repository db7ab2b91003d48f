# r05b: xxh32 quad kernel + worker changes: GPU tests (xxh32, single calls, frames), batch-hash rate,
# SQ counters of the parse and exec kernels (262 144 blocks)
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "xxh32 or single_call or frame or checksum" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/probe_xxh_batch.py > $O/xxh_batch.log 2>&1 || { tail -20 $O/xxh_batch.log; exit 1; }
cat $O/xxh_batch.log
NBLK=262144 DECS=rows REPS=1 bash tools/pmc_groups.sh $O/pmc_parse rows_parse tools/pmc/sq_parse2.txt tools/probe_rows.py || exit 1
NBLK=262144 DECS=rows REPS=1 bash tools/pmc_groups.sh $O/pmc_exec rows_exec tools/pmc/sq_parse2.txt tools/probe_rows.py || exit 1
