# r05as: host XXH32 rate by memory kind (pinned staging vs huge pages vs 4 KiB pages)
export TMPDIR=/tmp
O=gpurun_out/r05as
mkdir -p $O
timeout -k 10 200 python3 -u tools/probe_hash_mem.py > $O/hash_mem.log 2>&1 || { tail -20 $O/hash_mem.log; exit 1; }
grep -v amdgpu $O/hash_mem.log
