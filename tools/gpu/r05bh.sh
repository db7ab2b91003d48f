# r05bh: the default bench under rocprofv3 kernel-trace stats on the final tree (segmented parse, split-table linked passes)
export TMPDIR=/tmp
O=gpurun_out/r05bh
mkdir -p $O
cd /tmp && timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.log || { tail -20 $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
head -c 300 $GRAFT_REPO_ROOT/$O/bench_prof.json; echo
