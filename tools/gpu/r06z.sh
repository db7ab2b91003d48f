# r06z: block order and prefix sizes of the row decoder (probe_order.py) under
# the kernel trace: the parse / execution kernels' ramp + tail
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
cd /tmp && REPS=2 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o kt --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_order.py > $GRAFT_REPO_ROOT/$O/order.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/order.log; exit 1; }
cd $GRAFT_REPO_ROOT
cat $O/order.log | grep -v '^{'
f=$(find $O/kt -name "kt_kernel_trace.csv" | head -1)
python3 tools/dispatch_seq.py $f > $O/dispatches.txt
cat $O/dispatches.txt
rm -rf $O/kt
