# r04k: worker with one-round-trip request fields, record sizes from LDS; probe + single-call tests + per-call latency
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 90 python3 -u tools/probe_worker.py > $O/probe_worker.log 2>&1 || { cat $O/probe_worker.log; exit 1; }
cat $O/probe_worker.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -k "single_call" --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests_single.log 2>&1 || { tail -40 $O/tests_single.log; exit 1; }
tail -3 $O/tests_single.log
timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_worker.log 2>&1 && LZ4M_WORKER=0 timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_launch.log 2>&1
tail -12 $O/probe_c1_worker.log $O/probe_c1_launch.log
