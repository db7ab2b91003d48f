# r05y: config 4's hash-following decode timeline (decode launch ends vs host hash progress) at
# 16 (default), 64 and 4 block-ordered launches
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
for k in 16 64 4; do
  FOLLOW_CHUNKS=$k timeout -k 10 300 python3 -u tools/probe_c4_timeline.py > $O/timeline_$k.log 2>&1 || { tail -20 $O/timeline_$k.log; exit 1; }
  grep -v amdgpu $O/timeline_$k.log
done
bash tools/gpu/r05z.sh
