#!/bin/bash
# dev: the whole GPU suite, then the default bench
REPO=/root/repo
cd $REPO
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?
echo "bench rc=$rc2"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc2
