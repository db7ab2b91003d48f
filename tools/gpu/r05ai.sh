# r05ai: hist decoder -- the chain of sequence starts by a serial readlane walk (swalk) vs pointer
# jumping (head): 4 MiB blocks at 32 / 2048 per launch, 64 KiB blocks at 16 384; hist tests with swalk
export TMPDIR=/tmp
O=gpurun_out/r05ai
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/swalk/_lz4m.so LZ4M_DECODER=hist timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "decompress" > $O/hist_tests.log 2>&1 || { tail -30 $O/hist_tests.log; exit 1; }
tail -1 $O/hist_tests.log
for V in swalk head swalkb headb; do
  L=$PWD/tools/_abv/${V%b}/_lz4m.so; [ "${V%b}" = head ] && L=$PWD/python-lz4_amd/lz4/_lz4m.so
  LZ4M_LIB=$L timeout -k 10 300 python3 -u tools/probe_hist_big.py > $O/big_$V.log 2>&1 || { tail -20 $O/big_$V.log; exit 1; }
  echo "$V: $(grep -v amdgpu $O/big_$V.log | tr '\n' ' ')"
  LZ4M_LIB=$L DECS=hist NBLK=16384 REPS=3 timeout -k 10 200 python3 tools/probe_rows.py > $O/p64k_$V.log 2>&1 || { tail -20 $O/p64k_$V.log; exit 1; }
  echo "$V 64K: $(grep -o '"silesia/hist": {[^}]*}' $O/p64k_$V.log)"
done
