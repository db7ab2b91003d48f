# r04h: single-call worker debug probe (bounded waits), then the single-call tests
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 60 python3 -u tools/probe_worker.py 2>&1 | tee $O/probe_worker.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -k "single_call" --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests_single.log 2>&1 || { tail -40 $O/tests_single.log; exit 1; }
tail -3 $O/tests_single.log
timeout -k 10 120 python3 -u tools/probe_c1.py 2>&1 | tee $O/probe_c1_worker.log
