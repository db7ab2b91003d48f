# r04ae: lone-block decoder decodes into LDS (capacity <= 64 KiB): tests + per-call latency (random and compressible)
export TMPDIR=/tmp
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_codec.py -m gpu -x -q -k "single or solo or decompress" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -u tools/probe_c1.py > $O/probe_c1_worker.log 2>&1 && LZ4M_WORKER=0 timeout -k 10 200 python3 -u tools/probe_c1.py > $O/probe_c1_launch.log 2>&1
cat $O/probe_c1_worker.log $O/probe_c1_launch.log | grep -v amdgpu
