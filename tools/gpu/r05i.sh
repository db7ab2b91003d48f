# r05i: what each phase of the row executor costs -- timing probes that remove one phase each
# (WRONG output on purpose, LZ4M_ROWS_XP): 16 one pass without scans, 32 no literal puts,
# 64 no flush stores, 128 no match copies (scans kept), 256 no rebase copy
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1 || { tail -5 $O/probe_$n.log; exit 1; }; echo "== $n $(grep 'silesia rows' $O/probe_$n.log | head -1)"; }
for v in xp0 xp16 xp32 xp64 xp128 xp256; do run $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
run xp0b LZ4M_LIB=$PWD/tools/_abv/xp0/_lz4m.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "compress or dict or frame or linked or single_call or golden or pcompress or parallel" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/cmp_tests.log 2>&1 || { tail -30 $O/cmp_tests.log; exit 1; }
tail -2 $O/cmp_tests.log
pcr() { n=$1; shift; env "$@" NBLK=131072 KINDS=silesia,text,records REPS=3 MODES=exact timeout -k 10 300 python3 -u tools/prof_compress.py > $O/pc_$n.log 2>&1 || { tail -5 $O/pc_$n.log; exit 1; }; echo "== $n"; grep -v "^{" $O/pc_$n.log | grep -v amdgpu; }
for v in t0 t64 t96 t128 t257; do pcr $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
pcr main
