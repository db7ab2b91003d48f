# r04b: first run of the block-resident decoder -- focused parity tests, then
# decode-rate probe (resident vs rows) and its kernel statistics
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -v -k "resident" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_resident.log 2>&1 || { tail -40 $O/tests_resident.log; exit 1; }
tail -3 $O/tests_resident.log
NBLK=262144 DECS=resident,rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_262k.log 2>&1 || { tail -20 $O/probe_262k.log; exit 1; }
cat $O/probe_262k.log
NBLK=262144 DECS=resident,rows REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 -u tools/probe_rows.py > $O/probe_262k_prof.log 2>&1 || { tail -20 $O/probe_262k_prof.log; exit 1; }
find $O/kt -type f ! -name "*kernel_stats.csv" -delete
python3 -c "import csv;[print(r[0][:50],r[1],float(r[3])/1e6) for r in csv.reader(open(\"$O/kt/kt_kernel_stats.csv\")) if r[0]!=\"Name\"]"
LZ4M_LIB=$PWD/tools/_abv/prof/_lz4m.so NB=262144 timeout -k 10 300 python3 -u tools/prof_res.py > $O/prof_res.log 2>&1 || { tail -20 $O/prof_res.log; exit 1; }
cat $O/prof_res.log
