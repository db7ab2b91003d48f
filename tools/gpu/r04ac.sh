# r04ac: A/B -- rows decoder with the parse of chunk c+1 overlapped with the execution of chunk c (LZ4M_ROWS_OVERLAP) and a capped executor (LZ4M_ROWS_EXEC_WAVES)
export TMPDIR=/tmp
O=gpurun_out/r04ac
mkdir -p $O
LZ4M_ROWS_OVERLAP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "large_batch or rows" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_overlap4.log 2>&1 || { tail -30 $O/tests_overlap4.log; exit 1; }
tail -1 $O/tests_overlap4.log
run() { env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 400 python3 -u tools/probe_rows.py > $O/probe_$(echo "$@" | tr ' =' '__').log 2>&1; echo "== $@"; grep -v amdgpu $O/probe_$(echo "$@" | tr ' =' '__').log | grep rows | head -1; }
run LZ4M_ROWS_OVERLAP=0
run LZ4M_ROWS_OVERLAP=2
run LZ4M_ROWS_OVERLAP=4
run LZ4M_ROWS_OVERLAP=4 LZ4M_ROWS_EXEC_WAVES=16
run LZ4M_ROWS_OVERLAP=8 LZ4M_ROWS_EXEC_WAVES=16
run LZ4M_ROWS_OVERLAP=0 LZ4M_ROWS_EXEC_WAVES=16
