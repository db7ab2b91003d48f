# r04o: the first single-call compress of fresh processes
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
for a in "70000 70000" "70064 70000" "70000 65809" "70000 70000 torch"; do
  timeout -k 10 60 python3 -u tools/probe_first.py $a >> $O/probe_first.log 2>&1 || { cat $O/probe_first.log; exit 1; }
done
cat $O/probe_first.log
