# r06zm: the PMC traffic passes keyed to the final decoder sources
# (profiles/pmc_decompress.json, so the round-end bench line carries
# roofline.traffic) and the bench under the kernel trace
export TMPDIR=/tmp
O=gpurun_out/r06zm
mkdir -p $O
PMC_QUICK=1 timeout -k 10 900 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
head -c 700 $O/pmc/pmc_decompress.json; echo
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.log || { tail -20 $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
head -c 300 $O/bench_prof.json; echo
