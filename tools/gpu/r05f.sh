# r05f: VALU issue rates (micro), single-call worker lifetime 1 ms vs 5 ms (per-call latency and a
# batched launch beside a single-call loop), compressor probes -- exact parse without output stores
# (timing only, wrong bytes), the parallel parse with B's loads after A's walk -- then the full GPU
# suite (session-end worker check)
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 120 tools/micro/valu_rate.bin > $O/valu_rate.log 2>&1 || { tail -5 $O/valu_rate.log; exit 1; }
cat $O/valu_rate.log
c1() { n=$1; shift; env "$@" N=1000 timeout -k 10 120 python3 -u tools/probe_c1.py > $O/c1_$n.log 2>&1 || { tail -5 $O/c1_$n.log; exit 1; }; echo "== c1 $n: $(head -1 $O/c1_$n.log)"; }
bs() { n=$1; shift; env "$@" timeout -k 10 200 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q -s -k "beside_single_call" --timeout 150 --timeout-method thread -p no:cacheprovider > $O/beside_$n.log 2>&1 || { tail -30 $O/beside_$n.log; exit 1; }; echo "== beside $n: $(grep 'batched decode' $O/beside_$n.log)"; }
c1 life1
c1 life5 LZ4M_LIB=$PWD/tools/_abv/life5/_lz4m.so
bs life1
bs life5 LZ4M_LIB=$PWD/tools/_abv/life5/_lz4m.so
pcr() { n=$1; shift; env "$@" NBLK=131072 KINDS=silesia,text,records REPS=3 timeout -k 10 300 python3 -u tools/prof_compress.py > $O/pc_$n.log 2>&1 || { tail -5 $O/pc_$n.log; exit 1; }; echo "== $n"; grep -v "^{" $O/pc_$n.log | grep -v amdgpu; }
pcr base0
pcr cxp1 NOCHECK=1 MODES=exact LZ4M_LIB=$PWD/tools/_abv/cxp1/_lz4m.so
pcr pco1 MODES=parallel LZ4M_LIB=$PWD/tools/_abv/pco1/_lz4m.so
pcr base1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
