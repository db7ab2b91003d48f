# r05aa: config 4's block-ordered decode launches on the row decoder (forced) instead of the
# one-wavefront-per-block decoder: per-launch latency of 4 MiB blocks at 1, 8, 16, 64 launches
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
for k in 1 16 64 8; do
  DECODER=rows FOLLOW_CHUNKS=$k timeout -k 10 300 python3 -u tools/probe_c4_timeline.py > $O/timeline_rows_$k.log 2>&1 || { tail -20 $O/timeline_rows_$k.log; exit 1; }
  grep -v amdgpu $O/timeline_rows_$k.log
done
