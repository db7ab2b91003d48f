# r04ah: single-call tests after the worker's memory option was removed
export TMPDIR=/tmp
O=gpurun_out/r04ah
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_codec.py -m gpu -x -q -k "single or solo or many_threads" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
