# r06f: small executor cuts -- h2 (nok == 0 fast path for the row take count,
# the next length-byte sum inside parse_round), mo (+ both row sums
# interleaved), mou (+ unsigned in-block offsets) against h1 (the committed
# tree): 1 M-block probes, alternating
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
for i in 1 2; do
  run h1_$i LZ4M_LIB=$PWD/tools/_abv/h1/_lz4m.so
  run h2_$i LZ4M_LIB=$PWD/tools/_abv/h2/_lz4m.so
  run mo_$i LZ4M_LIB=$PWD/tools/_abv/mo/_lz4m.so
  run mou_$i LZ4M_LIB=$PWD/tools/_abv/mou/_lz4m.so
done
