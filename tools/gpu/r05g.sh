# r05g: the test of the next position merged into the search step (exact compressor): the
# compressor / frame / dict GPU tests, exact-parse timing with and without it; then PC sampling of the row decoder (which instructions of rows_exec / rows_parse the
# waves sit on, and why) -- list the box's PC-sampling configurations first
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 120 tools/micro/valu_rate.bin > $O/valu_rate.log 2>&1 || { tail -5 $O/valu_rate.log; exit 1; }
grep -E "cndmask|add_u32_e64|or3|v_and|v_add_u32 " $O/valu_rate.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "compress or dict or frame or linked or single_call or golden or pcompress or parallel" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/cmp_tests.log 2>&1 || { tail -30 $O/cmp_tests.log; exit 1; }
tail -2 $O/cmp_tests.log
pcr() { n=$1; shift; env "$@" NBLK=131072 KINDS=silesia,text,records REPS=3 MODES=exact timeout -k 10 300 python3 -u tools/prof_compress.py > $O/pc_$n.log 2>&1 || { tail -5 $O/pc_$n.log; exit 1; }; echo "== $n"; grep -v "^{" $O/pc_$n.log | grep -v amdgpu; }
pcr tnm1
pcr tnm0 LZ4M_LIB=$PWD/tools/_abv/tnm0/_lz4m.so
pcr tnm1b
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "rows or auto" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -2 $O/dec_tests.log
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
run head0
run ends0 LZ4M_LIB=$PWD/tools/_abv/ends0/_lz4m.so
run head1
timeout -k 10 90 rocprofv3 -L > $O/list.log 2>&1 || { tail -20 $O/list.log; exit 1; }
grep -i -B2 -A12 "pc.sampl\|pc_sampl" $O/list.log | head -60
pcs() { n=$1; shift; LZ4M_LIB=$PWD/tools/_abv/gline/_lz4m.so NBLK=262144 DECS=rows REPS=2 timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled "$@" -d $O/$n -o $n --output-format csv -- python3 -u tools/probe_rows.py > $O/$n.log 2>&1; rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; ls -R $O/$n | head; return $rc; }
pcs st --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576
rc=$?
# a configuration error (rc 1) only: no second GPU step after a crash or a time limit
if [ $rc -eq 1 ]; then pcs ht --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 10; fi
