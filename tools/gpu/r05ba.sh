# r05ba: segmented large-block parallel parse (lz4m_pcompress_large_batch): validity, then config-4 A/B
export TMPDIR=/tmp
O=gpurun_out/r05ba
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread \
  -k "parallel_parse or parallel" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "LZ4M_PC_SEG=1" "LZ4M_PC_SEG=1 LZ4M_PC_SEGHB=13" "LZ4M_PC_SEG=0"; do
  env $v timeout -k 10 300 python3 -u tools/probe_c4_cnochk.py > $O/cnochk.log 2>&1 || { tail -20 $O/cnochk.log; exit 1; }
  echo "$v"; grep -v amdgpu $O/cnochk.log | grep -v "launch alone"
  cp $O/cnochk.log "$O/cnochk_$(echo $v | tr ' =' '__').log"
done
