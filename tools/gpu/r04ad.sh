# r04ad: per-call latency on compressible blocks (worker and launch paths)
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
timeout -k 10 200 python3 -u tools/probe_c1.py > $O/probe_c1_worker.log 2>&1 && LZ4M_WORKER=0 timeout -k 10 200 python3 -u tools/probe_c1.py > $O/probe_c1_launch.log 2>&1
cat $O/probe_c1_worker.log $O/probe_c1_launch.log | grep -v amdgpu
