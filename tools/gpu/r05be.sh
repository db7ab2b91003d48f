# r05be: as r05bd, split table only where the u32 kernel does not fit at once: identity tests, then A/B on bench data
export TMPDIR=/tmp
O=gpurun_out/r05be
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread \
  -k "linked" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  LZ4M_SPEC_U17=$v DATA=bench BSIZES=65536 LZ4M_SPEC_VERBOSE=1 timeout -k 10 300 python3 -u tools/time_linked.py 256 silesia > $O/time_linked_u17_$v.log 2>&1 || { tail -20 $O/time_linked_u17_$v.log; exit 1; }
  echo "u17=$v"; grep -v amdgpu $O/time_linked_u17_$v.log | tail -9
done
