# r05aj: parallel-parse encoder -- sequence lookup by a DPP-reduced start mask (scat) vs the bpermute
# binary search (head): parallel-parse tests with scat, then A/B pairs at 262 144 blocks (same sizes digest)
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/scat/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "parallel" > $O/pc_tests.log 2>&1 || { tail -30 $O/pc_tests.log; exit 1; }
tail -1 $O/pc_tests.log
for V in scat head scatb headb; do
  L=$PWD/tools/_abv/${V%b}/_lz4m.so; [ "${V%b}" = head ] && L=$PWD/python-lz4_amd/lz4/_lz4m.so
  LZ4M_LIB=$L NB=262144 KINDS=silesia,text timeout -k 10 300 python3 -u tools/probe_pc.py > $O/pc_$V.log 2>&1 || { tail -20 $O/pc_$V.log; exit 1; }
  echo "$V: $(grep -v amdgpu $O/pc_$V.log | tr '\n' ' ')"
done
