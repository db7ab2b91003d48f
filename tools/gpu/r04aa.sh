# r04aa: A/B -- the exact compressor's test-next candidate from the ring when resident (LZ4M_TESTNEXT_RING)
export TMPDIR=/tmp
O=gpurun_out/r04aa
mkdir -p $O
LZ4M_LIB=tools/_abv/tnring/_lz4m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "compress" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_tnring.log 2>&1 || { tail -30 $O/tests_tnring.log; exit 1; }
tail -1 $O/tests_tnring.log
for i in 1 2; do
  NBLK=65536 KINDS=silesia,text,records MODES=exact REPS=3 timeout -k 10 300 python3 -u tools/prof_compress.py > $O/base_$i.log 2>&1
  NBLK=65536 KINDS=silesia,text,records MODES=exact REPS=3 LZ4M_LIB=tools/_abv/tnring/_lz4m.so timeout -k 10 300 python3 -u tools/prof_compress.py > $O/tnring_$i.log 2>&1
  echo "== base $i"; grep -v amdgpu $O/base_$i.log | tail -4; echo "== tnring $i"; grep -v amdgpu $O/tnring_$i.log | tail -4
done
