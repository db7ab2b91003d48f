# r06q: where the config-3 compressor's time goes, by ablation (timing only:
# NOLONG caps matches at 20 bytes -- valid blocks, worse ratio; NOCATCH skips
# the byte-wise catch-up; NOEMIT skips the encode -- blocks do not round-trip)
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
run() { v=$1; L=""; [ $v != head ] && L=$PWD/tools/_abv/$v/_lz4m.so
  LZ4M_LIB=$L NB=262144 KINDS=silesia,text,records timeout -k 10 300 python3 -u tools/probe_pc.py > $O/pc_$v.log 2>&1 || { tail -5 $O/pc_$v.log; exit 1; }
  echo "== $v"; cat $O/pc_$v.log | grep -v Warn; }
run pcbase && run pcnolong && run pcnocatch && run pcnoemit && run pcbase
