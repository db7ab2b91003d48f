# r05aq: bisect the VOP3-select sites (r05ao: wrong bytes with all five): the golden-corpus decode test
# per single-site build; stops at the first out-of-bounds fault, goes on after wrong output
export TMPDIR=/tmp
O=gpurun_out/r05aq
mkdir -p $O
for b in 1 2 4 8 16; do
  LZ4M_LIB=$PWD/tools/_abv/site$b/_lz4m.so timeout -k 10 200 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "test_decompress_matches_oracle and rows" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/site$b.log 2>&1
  rc=$?
  echo "site $b: rc=$rc $(tail -1 $O/site$b.log)"
  if grep -q "illegal memory access\|Memory access fault" $O/site$b.log; then echo "fault at site $b: stopping"; exit 1; fi
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
exit 0
