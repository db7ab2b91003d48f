# r06s: validation of the final tree (the encoder's permute lookup added after
# r06n; decoder sources unchanged, so r06n's PMC record stands) -- whole GPU
# suite, smoke, default bench, bench under the kernel trace; then the row
# decoder's finisher by data kind (kernel traces of the probe, 262 144 blocks)
export TMPDIR=/tmp
O=gpurun_out/r06s
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
for k in random runs text records; do
  cd /tmp && SEED=2026 KINDS=$k NBLK=262144 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$k -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/kt_$k.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_$k.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_$k -name "kt_kernel_stats.csv" | head -1)
  echo "== $k $(grep 'rows' $O/kt_$k.log | tail -1)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    for k in ("rows_parse", "rows_exec", "decompress_kernel"):
        if k in n:
            print(f"   {k:18s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
  rm -rf $O/kt_$k
done
