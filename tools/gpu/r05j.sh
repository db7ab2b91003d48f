# r05j: row executor copy-phase probes (WRONG output on purpose): 512 no long-match loop,
# 1024 no match puts, 2048 no match-source LDS reads; then the full default bench
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
for v in xp0 xp512 xp1024 xp2048; do run $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
timeout -k 10 1000 python3 -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.json
