# r05ap: the VOP3 select helpers against plain ternaries in isolation (no memory risk)
export TMPDIR=/tmp
O=gpurun_out/r05ap
mkdir -p $O
timeout -k 10 120 ./tools/micro/sel_check.bin > $O/sel_check.log 2>&1 || { tail -20 $O/sel_check.log; exit 1; }
cat $O/sel_check.log
