# r05at: decompress_host copies queued as their waits complete vs up front, per chunk size; its tests
export TMPDIR=/tmp
O=gpurun_out/r05at
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q -k "host" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/host_tests.log 2>&1 || { tail -30 $O/host_tests.log; exit 1; }
tail -1 $O/host_tests.log
timeout -k 10 400 python3 -u tools/probe_e2e.py > $O/e2e.log 2>&1 || { tail -20 $O/e2e.log; exit 1; }
grep -v amdgpu $O/e2e.log
