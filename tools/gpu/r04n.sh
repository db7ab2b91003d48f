# r04n: lz4m_compress_default on random blocks at capacities around the bound
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 120 python3 -u tools/probe_cdef.py > $O/probe_cdef.log 2>&1 || { cat $O/probe_cdef.log; exit 1; }
cat $O/probe_cdef.log
