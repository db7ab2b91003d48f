# r04ag: large-size byte identity -- exact compressor at 262 144 blocks (sampled vs the oracle), a 1 GiB frame vs the reference LZ4F_compressFrame
export TMPDIR=/tmp
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -k "large_batch_sampled or 1gib" --timeout 500 --timeout-method thread -p no:cacheprovider --durations=3 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -8 $O/tests.log
