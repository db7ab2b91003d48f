# r04af: persistent copy pool + the partition fix: large odd-size drop-in frames, frame API tests, drop-in config-4 probe
export TMPDIR=/tmp
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q -k "frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 -u tools/probe_c4_dropin.py > $O/c4_dropin.log 2>&1; grep -v amdgpu $O/c4_dropin.log | tail -6
