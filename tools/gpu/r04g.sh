# r04g: single-call persistent worker -- single-call tests (worker and launch modes),
# per-call probe with the worker and with LZ4M_WORKER=0
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -k "single_call" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_single.log 2>&1 || { tail -40 $O/tests_single.log; exit 1; }
tail -3 $O/tests_single.log
timeout -k 10 300 python3 -u tools/probe_c1.py > $O/probe_c1_worker.log 2>&1 || { tail -20 $O/probe_c1_worker.log; exit 1; }
cat $O/probe_c1_worker.log
LZ4M_WORKER=0 timeout -k 10 300 python3 -u tools/probe_c1.py > $O/probe_c1_launch.log 2>&1 || { tail -20 $O/probe_c1_launch.log; exit 1; }
cat $O/probe_c1_launch.log
