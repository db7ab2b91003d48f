# r05az: device frame decode with the follow launches split over three streams: tests, then config-4 A/B
export TMPDIR=/tmp
O=gpurun_out/r05az
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread -k "frame_decompress_device or frame_decompress" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1; do
  LZ4M_FOLLOW_SPLIT=$v timeout -k 10 300 python3 -u tools/probe_c4_timeline.py > $O/timeline_$v.log 2>&1 || { tail -20 $O/timeline_$v.log; exit 1; }
  echo "split=$v"; grep -v amdgpu $O/timeline_$v.log | grep -v "hash done at"
done
