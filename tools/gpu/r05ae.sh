# r05ae: config 4's exact compression (4 MiB blocks) split into block-ordered launches, one vs two streams
export TMPDIR=/tmp
O=gpurun_out/r05ae
mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_c4_cspans.py > $O/cspans.log 2>&1 || { tail -20 $O/cspans.log; exit 1; }
grep -v amdgpu $O/cspans.log
