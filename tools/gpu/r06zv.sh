# r06zv: the parallel-parse compressor's output staged in a 256-byte LDS ring
# per wave and flushed in whole 16-byte chunks (stg: 96 VGPRs with 48 B/lane of
# spills; stg4: 4 waves per SIMD, no spills) against the tree (cur); the
# round trip through the decoder checks every block
export TMPDIR=/tmp
O=gpurun_out/r06zv
mkdir -p $O
kt() { v=$1
  cd /tmp && NB=262144 KINDS=silesia,runs,random LZ4M_LIB=$GRAFT_REPO_ROOT/tools/_abv/$v/_lz4m.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$v -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_pc.py > $GRAFT_REPO_ROOT/$O/kt_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/kt_$v -name "kt_kernel_stats.csv" | head -1)
  echo "== $v"; grep 'parallel' $O/kt_$v.log | cut -c1-160
  rm -rf $O/kt_$v
}
kt cur && kt stg && kt stg4 && kt cur && kt stg && kt stg4
