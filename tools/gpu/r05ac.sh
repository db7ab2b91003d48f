# r05ac: huge-page result buffers + the 3-launch pipelined drop-in decode: frame GPU tests, the
# config-4 drop-in probe (pipeline traced), the follow decode at 4 launches, linked frame timing
export TMPDIR=/tmp
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "frame or host" > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 1; }
tail -2 $O/frame_tests.log
LZ4M_PIPE_TRACE=1 timeout -k 10 400 python3 -u tools/probe_c4_dropin.py > $O/c4_dropin.log 2>&1 || { tail -20 $O/c4_dropin.log; exit 1; }
grep -v amdgpu $O/c4_dropin.log
timeout -k 10 300 python3 -u tools/probe_c4_timeline.py > $O/timeline_4.log 2>&1 || { tail -20 $O/timeline_4.log; exit 1; }
grep -v amdgpu $O/timeline_4.log | grep -v "hash done at"
BSIZES=65536 LZ4M_SPEC_VERBOSE=1 timeout -k 10 300 python3 -u tools/time_linked.py 256 silesia > $O/time_linked.log 2>&1 || { tail -20 $O/time_linked.log; exit 1; }
grep -v amdgpu $O/time_linked.log
