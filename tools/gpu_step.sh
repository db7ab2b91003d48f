#!/bin/bash
cd /root/repo
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 200 --timeout-method thread -k "decompress" > gpurun_out/t1.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NBLK=262144 DECS=rows,lane,hist timeout -k 10 300 python -u tools/probe_rows.py > gpurun_out/p1.log 2>&1
rc2=$?
echo "probe rc=$rc2"; tail -5 gpurun_out/p1.log
exit $rc2
