# r06zr: validation of the final tree (the parse ring at absolute 64-byte lines) -- GPU suite, smoke, the
# default bench, the bench under rocprofv3 kernel-trace stats, and the PMC
# traffic passes keyed to the decoder sources (profiles/pmc_decompress.json)
export TMPDIR=/tmp
O=gpurun_out/r06zr
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
head -c 400 $O/bench.json; echo
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.log || { tail -20 $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
head -c 300 $O/bench_prof.json; echo
PMC_QUICK=1 timeout -k 10 900 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cat $O/pmc/pmc_decompress.json | head -c 600; echo
# the parse kernel's own write traffic (its 16-byte length-byte stores)
cd /tmp && SEED=2026 NBLK=262144 DECS=rows REPS=1 timeout -k 10 300 rocprofv3 --kernel-include-regex rows_parse --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$O/pmc_parse_w/p1 -o p1 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/pmc_parse_w.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/pmc_parse_w.log; exit 1; }
cd $GRAFT_REPO_ROOT && echo "-- rows_parse WRITE_SIZE (262 144 blocks x 2 launches)" && python3 tools/pmc_sum.py $O/pmc_parse_w rows_parse
