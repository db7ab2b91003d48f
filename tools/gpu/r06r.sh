# r06r: config-3 compressor encode -- the sequence of each output byte by one
# forward permute + a prefix max instead of a 6-step bpermute binary search
# (SCANSEQ), long matches counted 1 KiB per round trip instead of 256 B
# (WC16); parallel-parse suites on pcboth, probes (sizes digests must match)
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/pcboth/_lz4m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "parallel or pcompress or compress_many or frame" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_pcboth.log 2>&1 || { tail -30 $O/tests_pcboth.log; exit 1; }
tail -n 1 $O/tests_pcboth.log
run() { v=$1; L=""; [ $v != head ] && L=$PWD/tools/_abv/$v/_lz4m.so
  LZ4M_LIB=$L NB=262144 KINDS=silesia,text,records timeout -k 10 300 python3 -u tools/probe_pc.py > $O/pc_$v.log 2>&1 || { tail -5 $O/pc_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/pc_$v.log; }
run pcbase && run pcscan && run pcwc16 && run pcboth && run pcbase && run pcboth
