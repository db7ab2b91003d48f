# r03c: GPU suite on the new default (counted waits + paired parse), A/B of
# both changes with per-kernel times, phase split, SQ counters per sequence,
# counter calibration and the decoder's HBM traffic (calibrated method)
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for V in default p0 c0; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  tail -1 $O/probe_$V.log
done
LZ4M_LIB=$PWD/tools/_prof/_lz4m_rprof.so NB=262144 timeout -k 10 200 python3 -u tools/prof_rows.py > $O/rows_phases.log 2>&1 || exit $?
cat $O/rows_phases.log
DECS=rows NBLK=262144 REPS=1 timeout -k 10 400 bash tools/pmc_groups.sh $O/sq "rows_exec_kernel|rows_parse_kernel" tools/pmc/sq_exec.txt tools/probe_rows.py > $O/sq.log 2>&1 || exit $?
LZ4M_LIB=$PWD/tools/_abv/c0/_lz4m.so DECS=rows NBLK=262144 REPS=1 timeout -k 10 400 bash tools/pmc_groups.sh $O/sq_c0 "rows_exec_kernel|rows_parse_kernel" tools/pmc/sq_exec.txt tools/probe_rows.py > $O/sq_c0.log 2>&1 || exit $?
timeout -k 10 300 bash tools/pmc_cal.sh $O/cal > $O/cal.log 2>&1; echo cal=$?
CAL=$PWD/$O/cal/calibration.json timeout -k 10 900 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1; echo pmc=$?
cat $O/pmc/pmc_decompress.json
