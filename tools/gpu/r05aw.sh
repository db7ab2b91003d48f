# r05aw: device frame decode returns the slots when every block but the last is full (no gather): frame
# tests, then the config-4 no-checksum decode probe
export TMPDIR=/tmp
O=gpurun_out/r05aw
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "frame" > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 1; }
tail -1 $O/frame_tests.log
timeout -k 10 300 python3 -u tools/probe_c4_nochk.py > $O/nochk.log 2>&1 || { tail -20 $O/nochk.log; exit 1; }
grep -v amdgpu $O/nochk.log
