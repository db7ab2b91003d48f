# r05bg: row executor held to 6 waves per SIMD (80 VGPRs, 72 B/lane of spills) vs 5, A/B at 1 M blocks
export TMPDIR=/tmp
O=gpurun_out/r05bg
mkdir -p $O
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run w6 LZ4M_LIB=$PWD/tools/_abv/w6/_lz4m.so
run head
run w6b LZ4M_LIB=$PWD/tools/_abv/w6/_lz4m.so
run headb
