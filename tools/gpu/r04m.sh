# r04m: one random 64 KiB block's decode, per call, worker on and off
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 120 python3 -u tools/probe_slowdec.py > $O/probe_slowdec.log 2>&1 || { cat $O/probe_slowdec.log; exit 1; }
cat $O/probe_slowdec.log
