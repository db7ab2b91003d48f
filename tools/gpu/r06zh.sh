# r06zh: a plain 5.5 GB device copy beside the row decoder (tools/probe_concurrent.py)
export TMPDIR=/tmp
O=gpurun_out/r06zh
mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_concurrent.py > $O/concurrent.log 2>&1 || { tail -5 $O/concurrent.log; exit 1; }
cat $O/concurrent.log
