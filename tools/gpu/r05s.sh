# r05s: config-4 decode with the hash following (event wait releases the GIL), then the decoder's
# HBM traffic by PMC over the bench workload (profiles/pmc_decompress.json for roofline.traffic)
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 400 python3 -u tools/probe_c4_follow.py > $O/c4_follow.log 2>&1 || { tail -10 $O/c4_follow.log; exit 1; }
grep -v amdgpu $O/c4_follow.log
PMC_QUICK=1 bash tools/pmc_bench.sh $GRAFT_REPO_ROOT/$O/pmc || exit 1
cat $GRAFT_REPO_ROOT/$O/pmc/report.json | head -40
