export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03b/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
LZ4M_LIB=$PWD/tools/_prof/_lz4m_rprof.so NB=262144 timeout -k 10 200 python3 -u tools/prof_rows.py > gpurun_out/r03b/rows_phases.log 2>&1 && \
LZ4M_LIB=$PWD/tools/_prof/_lz4m_rprof.so NB=262144 timeout -k 10 200 python3 -u tools/prof_quad.py > gpurun_out/r03b/quad_phases.log 2>&1 && \
timeout -k 10 900 python -u bench.py > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b/kt -o kt -- python3 bench.py > gpurun_out/r03b/bench_under_rocprof.json 2> gpurun_out/r03b/bench_rocprof.err
rc2=$?; [ $rc2 -eq 0 ] && timeout -k 10 300 bash tools/pmc_cal.sh gpurun_out/r03b/cal > gpurun_out/r03b/cal.log 2>&1; echo cal=$?; echo rc=$rc2; cat gpurun_out/r03b/rows_phases.log gpurun_out/r03b/quad_phases.log; head -c 1200 gpurun_out/r03b/bench.json; exit $rc2
