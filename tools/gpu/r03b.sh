# r03b: GPU suite on HEAD, decoder A/B (per-kernel times), phase split, bench + its rocprofv3 stats
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 tools/micro/lds_align > $O/lds_align.log 2>&1 || exit $?
cat $O/lds_align.log
for V in default n1 p0 c0; do
  L=""; [ $V != default ] && L=$PWD/tools/_abv/$V/_lz4m.so
  LZ4M_LIB=$L DECS=rows NBLK=1048576 REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$V -o kt -- python3 tools/probe_rows.py > $O/probe_$V.log 2>&1 || exit $?
  tail -1 $O/probe_$V.log
done
LZ4M_LIB=$PWD/tools/_prof/_lz4m_rprof.so NB=262144 timeout -k 10 200 python3 -u tools/prof_rows.py > $O/rows_phases.log 2>&1 || exit $?
cat $O/rows_phases.log
(cd /tmp && DECS=rows NBLK=262144 REPS=1 timeout -s KILL 120 rocprofv3 --kernel-include-regex "rows_exec_kernel" --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d $GRAFT_REPO_ROOT/$O/lds_pmc -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_rows.py > $GRAFT_REPO_ROOT/$O/lds_pmc.log 2>&1); echo lds_pmc=$?
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
head -c 1500 $O/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/bench_rocprof.err
