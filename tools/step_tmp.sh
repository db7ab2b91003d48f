set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread -m gpu -k "compress or dict or linked or reference_bytes or block" > gpurun_out/t18.log 2>&1 || { tail -30 gpurun_out/t18.log; exit 1; }
tail -2 gpurun_out/t18.log
NBLK=16384 MODES=exact KINDS=silesia,text,records timeout -k 10 300 python -u tools/prof_compress.py > gpurun_out/pc18.log 2>&1 && grep -v json gpurun_out/pc18.log
LZ4M_LIB=tools/_prof/_lz4m_cprof.so KINDS=silesia,text,records timeout -k 10 300 python -u tools/prof_cphase.py > gpurun_out/cph.log 2>&1; cat gpurun_out/cph.log
if [ -n "$LINKED" ]; then timeout -k 10 300 python -u tools/time_linked.py 64 silesia text > gpurun_out/linked18.log 2>&1; cat gpurun_out/linked18.log; fi
