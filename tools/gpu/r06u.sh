# r06u: the config-3 compressor's long-match count at 4 bytes per lane for the
# first 256 bytes and 16 per lane (1 KiB per round trip) past them (WCHYB);
# parallel-parse suites on it, probes (sizes digests must match)
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/pchyb/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "parallel or pcompress or compress_many or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_pchyb.log 2>&1 || { tail -30 $O/tests_pchyb.log; exit 1; }
tail -n 1 $O/tests_pchyb.log
run() { v=$1; L=$PWD/tools/_abv/$v/_lz4m.so
  LZ4M_LIB=$L NB=262144 KINDS=silesia,text,runs timeout -k 10 300 python3 -u tools/probe_pc.py > $O/pc_$v.log 2>&1 || { tail -5 $O/pc_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/pc_$v.log; }
run pcb2 && run pchyb && run pcb2 && run pchyb
