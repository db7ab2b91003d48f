# r06o: 1280- against 1024-byte row histories (both with the round-6 parse) on
# the bench's own blocks (seed 2026, ratio 1.96) and the probe's (seed 7, 1.86):
# the r06n bench trace had the executor at 97.9 ms against r06g's 95.3
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
kt() { v=$1; seed=$2; L=""; [ $v != head ] && L=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so
  cd /tmp && LZ4M_LIB=$L SEED=$seed NBLK=1048576 DECS=rows REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_${v}_$seed -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/kt_${v}_$seed.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_${v}_$seed.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_${v}_$seed -name "kt_kernel_stats.csv" | head -1)
  echo "== $v seed $seed $(grep 'silesia rows' $O/kt_${v}_$seed.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    for k in ("rows_parse", "rows_exec", "decompress_kernel"):
        if k in n:
            print(f"   {k:18s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
  rm -rf $O/kt_${v}_$seed
}
kt head 2026 && kt h1024 2026 && kt head 2026 && kt h1024 2026 && kt head 7 && kt h1024 7
