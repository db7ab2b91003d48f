# r05ax: config-4 device frame compress without checksum: whole call vs the compression launch
export TMPDIR=/tmp
O=gpurun_out/r05ax
mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_c4_cnochk.py > $O/cnochk.log 2>&1 || { tail -20 $O/cnochk.log; exit 1; }
grep -v amdgpu $O/cnochk.log
