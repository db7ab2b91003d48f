# r05ay: windowed u16 table for the big-block parallel parse: validity per table, then config-4 A/B
export TMPDIR=/tmp
O=gpurun_out/r05ay
mkdir -p $O
for v in 0 12 13; do
  LZ4M_PC_LARGE=$v timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread \
    -k "parallel_parse_large or parallel_parse_valid" > $O/test_$v.log 2>&1 || { tail -30 $O/test_$v.log; exit 1; }
  tail -1 $O/test_$v.log
done
for v in 0 12 13; do
  LZ4M_PC_LARGE=$v timeout -k 10 300 python3 -u tools/probe_c4_cnochk.py > $O/cnochk_$v.log 2>&1 || { tail -20 $O/cnochk_$v.log; exit 1; }
  grep -v amdgpu $O/cnochk_$v.log
done
