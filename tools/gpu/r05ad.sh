# r05ad: the drop-in pipelined decode with downloads queued only after their launch ends; frame tests, drop-in probe
export TMPDIR=/tmp
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "frame or host" > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 1; }
tail -2 $O/frame_tests.log
LZ4M_PIPE_TRACE=1 timeout -k 10 400 python3 -u tools/probe_c4_dropin.py > $O/c4_dropin.log 2>&1 || { tail -20 $O/c4_dropin.log; exit 1; }
grep -v amdgpu $O/c4_dropin.log
