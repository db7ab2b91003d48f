# r06zy: 16-byte global loads by byte alignment (tools/micro/gload_align.hip)
set -e
O=gpurun_out/r06zy
mkdir -p $O
timeout -k 10 120 ./tools/_abv/gload_align > $O/gload_align.log 2>&1
cat $O/gload_align.log
