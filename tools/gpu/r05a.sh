# r05a: row executor timing probes (XP bits: 1 sync drain; 2,4,8 give wrong bytes -- timing only)
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n"; grep "silesia rows" $O/probe_$n.log | head -1; }
run base0
for v in xp1 xp3 xp7 xp15; do run $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
run base1
