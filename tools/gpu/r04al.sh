# r04al: ablation -- same-hash mask over 6 / 9 of the 12 hash bits (valid output, other sizes): the ballots' share of the time
export TMPDIR=/tmp
O=gpurun_out/r04al
mkdir -p $O
run() { n=$1; shift; env "$@" NB=262144 KINDS=silesia,text timeout -k 10 300 python3 -u tools/probe_pc.py > $O/probe_$n.log 2>&1 && echo "== $n" && grep -v amdgpu $O/probe_$n.log; }
run base0 && run eq6 LZ4M_LIB=$PWD/tools/_abv/eq6/_lz4m.so && run eq9 LZ4M_LIB=$PWD/tools/_abv/eq9/_lz4m.so && run base1
