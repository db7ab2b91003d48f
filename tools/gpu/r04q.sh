# r04q: lone-block compress output in LDS, LDS-typed literal reads and LDS bounce copy-out in the lone-block decoder
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_codec.py -m gpu -x -v -k "single_call or single or solo or linked or frame_is_reference" --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests_single.log 2>&1 || { tail -40 $O/tests_single.log; exit 1; }
tail -3 $O/tests_single.log
LZ4M_LIB=tools/_abv/wts/_lz4m.so timeout -k 10 120 python3 -u tools/probe_wts.py > $O/probe_wts.log 2>&1 || { cat $O/probe_wts.log; exit 1; }
cat $O/probe_wts.log
timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_worker.log 2>&1 && LZ4M_WORKER=0 timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_launch.log 2>&1
cat $O/probe_c1_worker.log $O/probe_c1_launch.log
LZ4M_SPEC_VERBOSE=1 timeout -k 10 180 python3 -u tools/time_linked.py 256 > $O/time_linked.log 2>&1
tail -30 $O/time_linked.log
LZ4M_WORKER_MEM=nc timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_worker_nc.log 2>&1 && LZ4M_WORKER_MEM=nc timeout -k 10 120 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q -k "single_call" --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests_single_nc.log 2>&1
cat $O/probe_c1_worker_nc.log; tail -2 $O/tests_single_nc.log
LZ4M_WORKER_MEM=nc LZ4M_LIB=tools/_abv/wts/_lz4m.so timeout -k 10 120 python3 -u tools/probe_wts.py > $O/probe_wts_nc.log 2>&1; cat $O/probe_wts_nc.log
