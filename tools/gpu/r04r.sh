# r04r: linked speculative compress, per-pass times: LDS-staged late passes (default) vs batched (LZ4M_SPEC_LDS=0) vs LDS only at <= 256 redo blocks
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
for v in 2048 0 256; do
  BSIZES=65536 LZ4M_SPEC_LDS=$v LZ4M_SPEC_VERBOSE=1 timeout -k 10 180 python3 -u tools/time_linked.py 256 > $O/time_linked_$v.log 2>&1 || { cat $O/time_linked_$v.log; exit 1; }
  echo "== LZ4M_SPEC_LDS=$v"; grep -v amdgpu $O/time_linked_$v.log | head -14
done
