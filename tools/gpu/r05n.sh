# r05n: the parallel parse with the ordered LDS exchange (LZ4M_PC_XCHG) and the lane-order
# self-test: compressor suites + self-test, parallel-parse A/B, then the default bench
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
true
tail -2 $O/cmp_tests.log
pcr() { n=$1; shift; env "$@" NBLK=131072 KINDS=silesia,text,records REPS=3 MODES=parallel timeout -k 10 300 python3 -u tools/prof_compress.py > $O/pc_$n.log 2>&1 || { tail -5 $O/pc_$n.log; exit 1; }; echo "== $n"; grep -v "^{" $O/pc_$n.log | grep -v amdgpu; }
pcr pcx1
pcr pcx0 LZ4M_LIB=$PWD/tools/_abv/pcx0/_lz4m.so
pcr pcx1b
timeout -k 10 1000 python3 -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.json
