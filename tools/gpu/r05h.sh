# r05h: exact compressor -- output staged in LDS (LZ4M_CMP_STAGE) and the merged test of the
# next position (LZ4M_CMP_TNMERGE), bit-exactness on the compressor / frame / dict suites, then a
# 2x2 A/B on one box (all four built the same way); row executor LDS / VALU counters
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "compress or dict or frame or linked or single_call or golden or pcompress or parallel" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/cmp_tests.log 2>&1 || { tail -30 $O/cmp_tests.log; exit 1; }
tail -2 $O/cmp_tests.log
pcr() { n=$1; shift; env "$@" NBLK=131072 KINDS=silesia,text,records REPS=3 MODES=exact timeout -k 10 300 python3 -u tools/prof_compress.py > $O/pc_$n.log 2>&1 || { tail -5 $O/pc_$n.log; exit 1; }; echo "== $n"; grep -v "^{" $O/pc_$n.log | grep -v amdgpu; }
for v in cb ct cs cm cb; do pcr $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
pcr main
NBLK=262144 DECS=rows REPS=1 bash tools/pmc_groups.sh $O/pmc_exec rows_exec tools/pmc/sq_exec_lds.txt tools/probe_rows.py || exit 1
python3 tools/pmc_sum.py $O/pmc_exec rows_exec
