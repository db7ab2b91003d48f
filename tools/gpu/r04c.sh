# r04c: resident decoder after the unrolled chunk loop: focused tests, rate
# probe (resident W=4, W=8, rows), kernel stats, phase split (W=4)
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "resident" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_resident.log 2>&1 || { tail -40 $O/tests_resident.log; exit 1; }
tail -2 $O/tests_resident.log
NBLK=262144 DECS=resident,rows REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_262k.log 2>&1 || { tail -20 $O/probe_262k.log; exit 1; }
grep -v "^{" $O/probe_262k.log
LZ4M_LIB=$PWD/tools/_abv/w8/_lz4m.so NBLK=262144 DECS=resident REPS=3 timeout -k 10 300 python3 -u tools/probe_rows.py > $O/probe_262k_w8.log 2>&1 || { tail -20 $O/probe_262k_w8.log; exit 1; }
grep -v "^{" $O/probe_262k_w8.log
LZ4M_LIB=$PWD/tools/_abv/prof/_lz4m.so NB=262144 timeout -k 10 300 python3 -u tools/prof_res.py > $O/prof_res.log 2>&1 || { tail -20 $O/prof_res.log; exit 1; }
cat $O/prof_res.log
NBLK=262144 DECS=resident REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 -u tools/probe_rows.py > $O/probe_262k_prof.log 2>&1 || { tail -20 $O/probe_262k_prof.log; exit 1; }
find $O/kt -type f ! -name "*kernel_stats.csv" -delete
python3 -c "import csv,glob;[print(r[0][:50],r[1],float(r[3])/1e6) for r in csv.reader(open(glob.glob('$O/kt/**/*kernel_stats.csv',recursive=True)[0])) if r[0]!='Name']"
