# r04p: where a lone-block call's time goes (LZ4M_WORKER_TS diagnostic build)
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
LZ4M_LIB=tools/_abv/wts/_lz4m.so timeout -k 10 120 python3 -u tools/probe_wts.py > $O/probe_wts.log 2>&1 || { cat $O/probe_wts.log && timeout -k 10 60 python3 -u tools/probe_slowdec.py > $O/probe_slowdec.log 2>&1; cat $O/probe_slowdec.log; exit 1; }
cat $O/probe_wts.log && timeout -k 10 60 python3 -u tools/probe_slowdec.py > $O/probe_slowdec.log 2>&1; cat $O/probe_slowdec.log
