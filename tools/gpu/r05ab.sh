# r05ab: what bounds the drop-in download -- copies into a fresh result bytes object (page faults)
# vs touched memory, huge pages, thread count; and the follow decode at 2 / 8 launches
export TMPDIR=/tmp
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_fault.py > $O/fault.log 2>&1 || { tail -20 $O/fault.log; exit 1; }
grep -v amdgpu $O/fault.log
for k in 2 8; do
  FOLLOW_CHUNKS=$k timeout -k 10 300 python3 -u tools/probe_c4_timeline.py > $O/timeline_$k.log 2>&1 || { tail -20 $O/timeline_$k.log; exit 1; }
  grep -v amdgpu $O/timeline_$k.log | grep -v "hash done at"
done
