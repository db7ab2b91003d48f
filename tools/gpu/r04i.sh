# r04i: HBM traffic of the block-resident decoder on the bench workload (FETCH_SIZE, WRITE_SIZE
# passes), to set beside the row decoder's (profiles/pmc_decompress.json)
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
LZ4M_DECODER=resident PMC_QUICK=1 PMC_KERNELS="rows_parse_kernel,res_exec_kernel,decompress_kernel<false, true>" \
  KRX="rows_parse_kernel|res_exec_kernel|decompress_kernel<false, true>" CAL=$PWD/profiles/traffic_calibration.json \
  timeout -k 10 900 bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
find $O/pmc -type f ! -name "*counter_collection.csv" ! -name "*.json" -delete
head -c 1200 $O/pmc/pmc_decompress.json; echo
