# r05ah: hist_decompress_kernel phase split on 4 MiB blocks (32 and 512 per launch) and 64 KiB blocks
export TMPDIR=/tmp
O=gpurun_out/r05ah
mkdir -p $O
LZ4M_LIB=$PWD/tools/_abv/prof/_lz4m.so KINDS=silesia BS=4194304 NB=32 timeout -k 10 300 python3 -u tools/prof_hist.py > $O/prof_4m_32.log 2>&1 || { tail -20 $O/prof_4m_32.log; exit 1; }
grep -v amdgpu $O/prof_4m_32.log
LZ4M_LIB=$PWD/tools/_abv/prof/_lz4m.so KINDS=silesia BS=4194304 NB=512 timeout -k 10 300 python3 -u tools/prof_hist.py > $O/prof_4m_512.log 2>&1 || { tail -20 $O/prof_4m_512.log; exit 1; }
grep -v amdgpu $O/prof_4m_512.log
LZ4M_LIB=$PWD/tools/_abv/prof/_lz4m.so KINDS=silesia NB=2048 timeout -k 10 300 python3 -u tools/prof_hist.py > $O/prof_64k.log 2>&1 || { tail -20 $O/prof_64k.log; exit 1; }
grep -v amdgpu $O/prof_64k.log
