# r06zt: what the exact compressor's output stores cost (cxns: literal, offset
# and token stores skipped, wrong output on purpose, timing only) against the tree
export TMPDIR=/tmp
O=gpurun_out/r06zt
mkdir -p $O
for v in cur cxns cur cxns; do
  NOCHECK=1 NBLK=65536 KINDS=silesia MODES=exact REPS=2 LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so timeout -k 10 300 python3 -u tools/prof_compress.py > $O/pc_$v.log 2>&1 || { tail -5 $O/pc_$v.log; exit 1; }
  echo "== $v $(tail -1 $O/pc_$v.log | cut -c1-300)"
done
