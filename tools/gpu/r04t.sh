# r04t: exact compressor phase split (LZ4M_COMPRESS_PROF build): batched silesia/random, single-call random
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
KINDS=silesia,random,text NB=16384 SINGLE=1 LZ4M_LIB=tools/_abv/cprof/_lz4m.so timeout -k 10 300 python3 -u tools/prof_cphase.py > $O/prof_cphase.log 2>&1 || { cat $O/prof_cphase.log; exit 1; }
cat $O/prof_cphase.log
