# r04e: rows decoder A/B -- non-temporal input/length loads (LZ4M_ROWS_NT) vs default,
# 1 M blocks (the config-2 size: L2 and Infinity-Cache behaviour at scale); then the full bench
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
NBLK=1048576 DECS=rows REPS=3 timeout -k 10 400 python3 -u tools/probe_rows.py > $O/probe_default.log 2>&1 || { tail -20 $O/probe_default.log; exit 1; }
grep -v "^{" $O/probe_default.log
LZ4M_LIB=$PWD/tools/_abv/nt/_lz4m.so NBLK=1048576 DECS=rows REPS=3 timeout -k 10 400 python3 -u tools/probe_rows.py > $O/probe_nt.log 2>&1 || { tail -20 $O/probe_nt.log; exit 1; }
grep -v "^{" $O/probe_nt.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
head -c 3000 $O/bench.json; echo
