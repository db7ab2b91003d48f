# r05m: the exact compressor's search step with one LDS exchange per lane (LZ4M_CMP_XCHG):
# byte identity on the compressor / frame / dict / single-call suites, then A/B with the merged-test
# thresholds (0, 64, 128, always)
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "compress or dict or frame or linked or single_call or golden or pcompress or parallel" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/cmp_tests.log 2>&1 || { tail -30 $O/cmp_tests.log; exit 1; }
tail -2 $O/cmp_tests.log
pcr() { n=$1; shift; env "$@" NBLK=131072 KINDS=silesia,text,records REPS=3 MODES=exact timeout -k 10 300 python3 -u tools/prof_compress.py > $O/pc_$n.log 2>&1 || { tail -5 $O/pc_$n.log; exit 1; }; echo "== $n"; grep -v "^{" $O/pc_$n.log | grep -v amdgpu; }
for v in x0 x1 x1t0 x1t128 x1t257; do pcr $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
