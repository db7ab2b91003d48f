# r05p: config-4 frame decode with the content hash following block-ordered decode launches:
# the device frame tests, then the 8 GiB probe (follow on / off)
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q -k "frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 1; }
tail -1 $O/frame_tests.log
timeout -k 10 400 python3 -u tools/probe_c4_follow.py > $O/c4_follow.log 2>&1 || { tail -10 $O/c4_follow.log; exit 1; }
grep -v amdgpu $O/c4_follow.log
timeout -k 10 400 python3 -u tools/probe_c4_dropin.py > $O/c4_dropin.log 2>&1 || { tail -10 $O/c4_dropin.log; exit 1; }
grep -v amdgpu $O/c4_dropin.log | tail -6
LZ4M_FRAME_FOLLOW=0 timeout -k 10 400 python3 -u tools/probe_c4_dropin.py > $O/c4_dropin_off.log 2>&1 || { tail -10 $O/c4_dropin_off.log; exit 1; }
grep -v amdgpu $O/c4_dropin_off.log | tail -6
