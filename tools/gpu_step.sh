#!/bin/bash
# dev: decoder tests, then kernel-trace stats of the decoders on the probe workload
REPO=/root/repo
cd $REPO
timeout -k 10 420 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 200 --timeout-method thread -k "decompress" > gpurun_out/t3.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t3.log
if [ $rc -ne 0 ]; then exit $rc; fi
OUT=$REPO/gpurun_out/prof3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
NBLK=1048576 DECS=rows REPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $REPO/tools/probe_rows.py > $OUT/probe.log 2>&1
rc=$?
echo "rc=$rc"; grep silesia $OUT/probe.log
exit $rc
