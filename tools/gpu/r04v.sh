# r04v: LDS-window parse with the next search step prefetched, LDS last-literal copy; tests, per-call, linked passes, phase split
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_codec.py -m gpu -x -q -k "single or solo or linked or frame_is_reference or compress" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_worker.log 2>&1 && LZ4M_WORKER=0 timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_launch.log 2>&1
cat $O/probe_c1_worker.log $O/probe_c1_launch.log
for v in 256 100000; do
  BSIZES=65536 LZ4M_SPEC_LDS=$v LZ4M_SPEC_VERBOSE=1 timeout -k 10 180 python3 -u tools/time_linked.py 256 > $O/time_linked_$v.log 2>&1 || { cat $O/time_linked_$v.log; exit 1; }
  echo "== LZ4M_SPEC_LDS=$v"; grep -v amdgpu $O/time_linked_$v.log | head -7
done
KINDS=silesia NB=16384 SINGLE=1 LZ4M_LIB=tools/_abv/cprof/_lz4m.so timeout -k 10 300 python3 -u tools/prof_cphase.py > $O/prof_cphase.log 2>&1; cat $O/prof_cphase.log
