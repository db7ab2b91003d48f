# r05ag: linked speculative passes on bench.py's config-4 sample (make_batch seed 77, 256 MiB)
export TMPDIR=/tmp
O=gpurun_out/r05ag
mkdir -p $O
DATA=bench BSIZES=65536 LZ4M_SPEC_VERBOSE=1 timeout -k 10 300 python3 -u tools/time_linked.py 256 silesia > $O/time_linked.log 2>&1 || { tail -20 $O/time_linked.log; exit 1; }
grep -v amdgpu $O/time_linked.log
