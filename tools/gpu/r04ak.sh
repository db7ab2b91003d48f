# r04ak: parallel-parse compressor, same-hash resolution by LDS probe (default) vs one ballot per hash bit (pc0)
export TMPDIR=/tmp
O=gpurun_out/r04ak
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -x -q -m gpu -k "parallel or pcompress or PARALLEL" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
NB=262144 KINDS=silesia,random,runs,text timeout -k 10 300 python3 -u tools/probe_pc.py > $O/probe_new0.log 2>&1 && grep -v amdgpu $O/probe_new0.log &&
LZ4M_LIB=$PWD/tools/_abv/pc0/_lz4m.so NB=262144 KINDS=silesia,random,runs,text timeout -k 10 300 python3 -u tools/probe_pc.py > $O/probe_old.log 2>&1 && grep -v amdgpu $O/probe_old.log &&
NB=262144 KINDS=silesia,random,runs,text timeout -k 10 300 python3 -u tools/probe_pc.py > $O/probe_new1.log 2>&1 && grep -v amdgpu $O/probe_new1.log
