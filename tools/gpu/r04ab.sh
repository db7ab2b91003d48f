# r04ab: single calls from four host threads at once
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -k "many_threads" --timeout 200 --timeout-method thread -p no:cacheprovider --durations=3 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -8 $O/tests.log
