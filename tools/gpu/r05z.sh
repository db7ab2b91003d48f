# r05z: the pipelined drop-in frame decode (upload / block-ordered decode / download + hash
# overlapped): its GPU tests, the frame tests, and the config-4 drop-in probe (pipelined vs
# sequential)
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "frame" > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 1; }
tail -2 $O/frame_tests.log
timeout -k 10 400 python3 -u tools/probe_c4_dropin.py > $O/c4_dropin.log 2>&1 || { tail -20 $O/c4_dropin.log; exit 1; }
grep -v amdgpu $O/c4_dropin.log
BSIZES=65536 LZ4M_SPEC_VERBOSE=1 timeout -k 10 300 python3 -u tools/time_linked.py 256 silesia > $O/time_linked.log 2>&1 || { tail -20 $O/time_linked.log; exit 1; }
grep -v amdgpu $O/time_linked.log
