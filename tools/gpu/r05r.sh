# r05r: 256-thread executor workgroups as default (decoder suites, A/B against 64), the config-4
# decode stage split, the default linked frame's passes
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_api.py -m gpu -x -q -k "decompress or decode or rows or auto" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run ewg256
run ewg64 LZ4M_LIB=$PWD/tools/_abv/ewg64/_lz4m.so
run ewg256b
run ewg64b LZ4M_LIB=$PWD/tools/_abv/ewg64/_lz4m.so
LZ4M_FRAME_FOLLOW=0 timeout -k 10 400 python3 -u tools/probe_c4_decode.py > $O/c4_stages.log 2>&1 || { tail -10 $O/c4_stages.log; exit 1; }
grep -v amdgpu $O/c4_stages.log
LZ4M_SPEC_VERBOSE=1 BSIZES=65536 timeout -k 10 300 python3 -u tools/time_linked.py 256 > $O/time_linked.log 2>&1 || { tail -10 $O/time_linked.log; exit 1; }
grep -v amdgpu $O/time_linked.log | tail -20
