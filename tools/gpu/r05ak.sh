# r05ak: final decoder sources -- HBM traffic by PMC passes over the bench workload, then the default
# bench under rocprofv3 kernel-trace stats
export TMPDIR=/tmp
O=gpurun_out/r05ak
mkdir -p $O
PMC_QUICK=1 bash tools/pmc_bench.sh $GRAFT_REPO_ROOT/$O/pmc || exit 1
head -c 600 $GRAFT_REPO_ROOT/$O/pmc/pmc_decompress.json; echo
cd /tmp && timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.log || { tail -20 $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
head -c 300 $GRAFT_REPO_ROOT/$O/bench_prof.json; echo
