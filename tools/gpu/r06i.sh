# r06i: where the row executor's L2 misses are served -- TCC read requests,
# those that reached DRAM, L2 hits and misses (262 144 blocks, rows_exec only)
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
cd /tmp && NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex rows_exec --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum -d $GRAFT_REPO_ROOT/$O/t1 -o p1 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/t1.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/t1.log; exit 1; }
cd /tmp && NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex rows_exec --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum -d $GRAFT_REPO_ROOT/$O/t2 -o p2 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/t2.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/t2.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/pmc_sum.py $O rows_exec | tee $O/tcc.txt
grep "silesia rows" $O/t1.log
