# r04f: drop-in config-4 calls with the pipelined host transfers; frame API GPU tests
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_api.log 2>&1 || { tail -30 $O/tests_api.log; exit 1; }
tail -2 $O/tests_api.log
GIB=8 timeout -k 10 600 python3 -u tools/probe_c4_dropin.py > $O/c4_dropin.log 2>&1 || { tail -20 $O/c4_dropin.log; exit 1; }
cat $O/c4_dropin.log
