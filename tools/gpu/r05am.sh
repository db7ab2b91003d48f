# r05am: VOP2 v_cndmask_b32 reading VCC -- is it slow on gfx950, and in which pattern?
export TMPDIR=/tmp
O=gpurun_out/r05am
mkdir -p $O
timeout -k 10 120 ./tools/micro/cndmask_rate.bin > $O/cndmask_rate.log 2>&1 || { tail -20 $O/cndmask_rate.log; exit 1; }
cat $O/cndmask_rate.log
