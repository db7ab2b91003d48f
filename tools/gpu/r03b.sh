export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
DECS=rows,quad NBLK=1048576 REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > gpurun_out/r03b/probe_rows_quad.log 2>&1 && \
timeout -k 10 900 python -u bench.py > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b/kt -o kt -- python3 bench.py > gpurun_out/r03b/bench_under_rocprof.json 2> gpurun_out/r03b/bench_rocprof.err
rc=$?; echo rc=$rc; cat gpurun_out/r03b/probe_rows_quad.log; head -c 1500 gpurun_out/r03b/bench.json; exit $rc
