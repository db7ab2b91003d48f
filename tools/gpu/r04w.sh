# r04w: lone-block compress copies its last literals from the staged block with all four waves
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_codec.py -m gpu -x -q -k "single or solo" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_worker.log 2>&1 && LZ4M_WORKER=0 timeout -k 10 120 python3 -u tools/probe_c1.py > $O/probe_c1_launch.log 2>&1
cat $O/probe_c1_worker.log $O/probe_c1_launch.log
LZ4M_LIB=tools/_abv/wts/_lz4m.so timeout -k 10 120 python3 -u tools/probe_wts.py > $O/probe_wts.log 2>&1; cat $O/probe_wts.log
KINDS=silesia NB=4096 SINGLE=1 LZ4M_LIB=tools/_abv/cprof/_lz4m.so timeout -k 10 300 python3 -u tools/prof_cphase.py > $O/prof_cphase.log 2>&1; cat $O/prof_cphase.log
