#!/bin/bash
# dev: decoder tests, phase profile, then kernel-trace stats of the decoders on the probe workload
REPO=/root/repo
cd $REPO
timeout -k 10 420 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 200 --timeout-method thread -k "decompress" > gpurun_out/t3.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t3.log
if [ $rc -ne 0 ]; then exit $rc; fi
LZ4M_LIB=$REPO/tools/_prof/_lz4m_rprof.so NB=262144 KINDS=silesia timeout -k 10 300 python -u tools/prof_rows.py > gpurun_out/rprof.log 2>&1
rc=$?; echo "prof rc=$rc"; cat gpurun_out/rprof.log | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
OUT=$REPO/gpurun_out/prof8
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
NBLK=1048576 DECS=rows,lane REPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $REPO/tools/probe_rows.py > $OUT/probe.log 2>&1
rc=$?
echo "rc=$rc"; grep silesia $OUT/probe.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open('/root/repo/gpurun_out/prof8/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('rows_','decompress_kernel', 'stage_dec')):
        print(r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e6)
PY
exit $rc
