# r04aj: rows decoder macro A/B at 1 M blocks (parse general-step threshold; history keep / room)
export TMPDIR=/tmp
O=gpurun_out/r04aj
mkdir -p $O
run() { n=$1; shift; env "$@" NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_$n.log 2>&1; echo "== $n"; grep -v amdgpu $O/probe_$n.log | grep "silesia rows" | head -1; }
run base0
for v in pma32 pma48 keep384 room384; do run $v LZ4M_LIB=$PWD/tools/_abv/$v/_lz4m.so; done
run base1
